/* Diagnostic (round 4): does a single-rank RCCL all-to-all of >= 1.6 GB return the data it
 * was given?  Torch-free: libnutexec only generates the column (nut_gen_column) and owns
 * the stream; RCCL is called directly, so a wrong result here is RCCL's, not the
 * library's exchange code (dist.cpp).  For each size: ncclAllToAllv in one call, the same
 * as grouped ncclSend / ncclRecv, and in 2^26-word rounds; the receive buffer is filled
 * with a marker first, copied back and compared word by word with the send buffer.
 *   build: gcc -O2 a2a_probe.c -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__
 *          -L nutdb_amd -lnutexec -L /opt/rocm/lib -lrccl -lamdhip64 */
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nutexec.h"

#define HIPOK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)
#define NCCLOK(x)                                                                \
  do {                                                                           \
    ncclResult_t e_ = (x);                                                       \
    if (e_ != ncclSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(e_)); \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

static void report(const char *mode, size_t n, const uint64_t *want, const uint64_t *got) {
  size_t bad = 0, first = (size_t)-1, last = 0;
  for (size_t i = 0; i < n; ++i)
    if (want[i] != got[i]) {
      if (!bad) first = i;
      last = i;
      ++bad;
    }
  if (bad)
    printf("%-10s n=%zu (%.3f GB): WRONG %zu words, first %zu (byte %zu) last %zu, got[first]=%016llx want %016llx\n",
           mode, n, n * 8e-9, bad, first, first * 8, last, (unsigned long long)got[first],
           (unsigned long long)want[first]);
  else
    printf("%-10s n=%zu (%.3f GB): exact\n", mode, n, n * 8e-9);
  fflush(stdout);
}

int main(int argc, char **argv) {
  nut_ctx *ctx = NULL;
  if (nut_ctx_create(0, &ctx)) {
    fprintf(stderr, "nut_ctx_create: %s\n", nut_last_error());
    return 2;
  }
  hipStream_t st;
  HIPOK(hipStreamCreate(&st));
  if (nut_ctx_set_stream(ctx, st)) return 2;
  ncclUniqueId id;
  NCCLOK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NCCLOK(ncclCommInitRank(&comm, 1, id, 0));
  /* 2^27 words = 2^30 bytes: 1.3e8 (1.040 GB) and 1.342e8 (1.0736 GB) sit just below it,
   * 1.3422e8 (1.07376 GB) and 1.35e8 just above */
  const double sizes[] = {1e8, 1.3e8, 1.342e8, 1.3422e8, 1.35e8, 1.5e8, 2e8, 2.7e8};
  const int nsizes = argc > 1 ? atoi(argv[1]) : (int)(sizeof sizes / sizeof sizes[0]);
  const size_t nmax = (size_t)sizes[nsizes - 1];
  uint64_t *send, *recv;
  HIPOK(hipMalloc((void **)&send, nmax * 8));
  HIPOK(hipMalloc((void **)&recv, nmax * 8));
  uint64_t *hw = (uint64_t *)malloc(nmax * 8), *hg = (uint64_t *)malloc(nmax * 8);
  if (!hw || !hg) return 2;
  for (int si = 0; si < nsizes; ++si) {
    const size_t n = (size_t)sizes[si];
    if (nut_gen_column(ctx, NUT_GEN_FULL_I64, 0x5eed + si, 0, 0, 0, 0, n, send)) return 2;
    HIPOK(hipStreamSynchronize(st));
    HIPOK(hipMemcpy(hw, send, n * 8, hipMemcpyDeviceToHost));
    for (int mode = 0; mode < 3; ++mode) {
      HIPOK(hipMemsetAsync(recv, 0xA5, n * 8, st));
      size_t c = n, z = 0;
      if (mode == 0) {
        NCCLOK(ncclAllToAllv(send, &c, &z, recv, &c, &z, ncclUint64, comm, st));
      } else if (mode == 1) {
        NCCLOK(ncclGroupStart());
        NCCLOK(ncclSend(send, n, ncclUint64, 0, comm, st));
        NCCLOK(ncclRecv(recv, n, ncclUint64, 0, comm, st));
        NCCLOK(ncclGroupEnd());
      } else {
        const size_t ch = (size_t)1 << 27;  /* 2^30-byte rounds: the largest that stays exact? */
        for (size_t o = 0; o < n; o += ch) {
          size_t cc = n - o < ch ? n - o : ch, d = o;
          NCCLOK(ncclAllToAllv(send, &cc, &d, recv, &cc, &d, ncclUint64, comm, st));
        }
      }
      HIPOK(hipStreamSynchronize(st));
      HIPOK(hipMemcpy(hg, recv, n * 8, hipMemcpyDeviceToHost));
      report(mode == 0 ? "alltoallv" : mode == 1 ? "send/recv" : "rounds2^27", n, hw, hg);
    }
  }
  NCCLOK(ncclCommDestroy(comm));
  nut_ctx_destroy(ctx);
  printf("a2a_probe done\n");
  return 0;
}
