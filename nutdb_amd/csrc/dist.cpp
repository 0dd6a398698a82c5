// dist.cpp — multi-GPU execution inside the C ABI (nut_dist_*).
//
// A nut_dist is P ranks, one GPU each.  Its exchanges are RCCL collectives on each
// member's stream (ncclAllGather for the small per-rank headers, ncclAllToAllv for the
// records: xGMI is a full point-to-point mesh, so one all-to-all uses every link at once),
// or — for nut_dist_create_virtual — device copies between P members sharing one GPU,
// so that the same partition / exchange / merge code runs with P > 1 on a single device.
//
// RCCL is resolved with dlopen on the first nut_dist_create*: the single-GPU entry points
// never load it.  By soname ("librccl.so.1"), so a process that already holds an RCCL
// (torch's) reuses that copy and its HIP runtime instead of loading a second one.
//
// Every collective call starts with an all-gather of a small header that carries each
// rank's status, so a rank whose local step failed fails the call on every rank instead
// of leaving the others blocked in an all-to-all.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "sort.hpp"

using namespace nut;

namespace {

// ------------------------------------------------------------------ RCCL entry points
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllToAllv) all_to_allv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  std::string load_error;
};

Rccl g_rccl;
std::once_flag g_rccl_once;

template <class F>
bool bind(void *h, const char *name, F &fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

const Rccl *rccl() {
  std::call_once(g_rccl_once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char *e = dlerror();
      g_rccl.load_error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    Rccl r;
    if (!bind(h, "ncclGetUniqueId", r.get_unique_id) || !bind(h, "ncclCommInitRank", r.comm_init_rank) ||
        !bind(h, "ncclCommInitAll", r.comm_init_all) || !bind(h, "ncclCommDestroy", r.comm_destroy) ||
        !bind(h, "ncclAllGather", r.all_gather) || !bind(h, "ncclAllToAllv", r.all_to_allv) ||
        !bind(h, "ncclGetErrorString", r.error_string) || !bind(h, "ncclGroupStart", r.group_start) ||
        !bind(h, "ncclGroupEnd", r.group_end)) {
      g_rccl.load_error = "librccl.so.1 lacks an entry point nut_dist needs";
      return;
    }
    g_rccl = r;
  });
  return g_rccl.all_to_allv ? &g_rccl : nullptr;
}

nut_status rccl_fail(const Rccl *r, ncclResult_t e, const char *what) {
  return fail(NUT_ERR_HIP, std::string(what) + ": " + (r ? r->error_string(e) : "RCCL") + " (" +
                               std::to_string((int)e) + ")");
}

// ------------------------------------------------------------------ virtual ranks
// P members on one device: a post-and-copy exchange between threads.  A member posts its
// send buffer once its stream has drained, every member copies its parts out of the
// others' buffers on its own stream, and nobody leaves before all copies are complete.
struct Hub {
  std::mutex mu;
  std::condition_variable cv;
  int n = 0, arrived = 0;
  uint64_t generation = 0;
  struct Post {
    const uint64_t *send = nullptr;
    const size_t *count = nullptr, *displ = nullptr;  // words, per destination
    size_t words = 0;                                  // all-gather: words per rank
  };
  std::vector<Post> post;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != g; });
    }
  }
};

}  // namespace

struct nut_dist {
  enum Mode { kRcclAll, kRcclRank, kVirtual } mode = kRcclAll;
  int nranks = 1, first_rank = 0;
  const Rccl *r = nullptr;
  Hub hub;
  struct Member {
    int rank = 0;
    nut_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    Scratch hdr_dev;                  // headers: this rank's and the all-gathered ones
    uint64_t *hdr_host = nullptr;     // pinned, kHdrBytes: the all-gathered headers
    uint64_t *hdr_send = nullptr;     // pinned, kHdrWords + kSamples words: this rank's header, sample positions
    Scratch buf[10];                  // send / receive / output buffers of the calls
  };
  std::vector<Member> m;
};

namespace {

constexpr int kMaxRanks = 64;  // nut_groups_partition / nut_partition_i64 bound
constexpr size_t kHdrWords = 2 + 2 * kMaxRanks;
constexpr size_t kHdrBytes = kHdrWords * kMaxRanks * 8;
constexpr int kSamples = 4096;  // sample sort: strided samples per rank
constexpr uint64_t kSampleWords = 2 + kSamples;  // one rank's all-gathered [status, has keys, samples]
constexpr uint64_t kSortFlip = 1ull << 63;  // int64 order -> unsigned order

using Member = nut_dist::Member;

uint64_t *buf(Member &mb, int i) { return (uint64_t *)mb.buf[i].ptr; }
nut_status reserve(Member &mb, int i, uint64_t words) { return mb.buf[i].reserve(std::max<uint64_t>(words, 1) * 8); }

// all-gather of `words` words from every rank: recv[q * words + i]
nut_status allgather(nut_dist *d, int l, const uint64_t *send, uint64_t *recv, size_t words) {
  Member &mb = d->m[l];
  hipStream_t s = mb.ctx->stream;
  if (d->mode != nut_dist::kVirtual) {
    ncclResult_t e = d->r->all_gather(send, recv, words, ncclUint64, mb.comm, s);
    (void)hipGetLastError();  // RCCL leaves stale HIP errors in this thread's slot
    return e == ncclSuccess ? NUT_OK : rccl_fail(d->r, e, "ncclAllGather");
  }
  Hub &h = d->hub;
  NUT_HIP(hipStreamSynchronize(s));
  h.post[l] = Hub::Post{send, nullptr, nullptr, words};
  h.barrier();
  hipError_t e = hipSuccess;
  for (int q = 0; q < d->nranks && e == hipSuccess; ++q)
    if (words) e = hipMemcpyAsync(recv + (size_t)q * words, h.post[q].send, words * 8, hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  h.barrier();  // the senders' buffers stay untouched until every copy is done
  return e == hipSuccess ? NUT_OK : hip_fail(e, "nut_dist (virtual) all-gather");
}

// RCCL all-to-all rounds move at most this many words per (sender, receiver) pair.  On
// RCCL 2.27.7 / ROCm 7.2 one P2P transfer of more than 2^30 bytes leaves everything after
// its first half unwritten (ncclAllToAllv and grouped ncclSend / ncclRecv alike; 134,200,000
// words exact, 134,220,000 wrong — the torch-free probe scripts/diag/a2a_probe.c,
// profiles/r04/dist/), so no pair moves more than half that limit per round
constexpr size_t kRcclP2PMaxBytes = size_t(1) << 30;
constexpr size_t kA2AChunk = kRcclP2PMaxBytes / 2 / sizeof(uint64_t);  // 2^26 words = 2^29 bytes
static_assert(kA2AChunk * sizeof(uint64_t) < kRcclP2PMaxBytes, "a round's transfer stays under RCCL's limit");

// the largest (sender, receiver) cell of an all-gathered count matrix: rank q's count for
// receiver r at all[q * w + off + r], times `mul` words per count
size_t max_cell(const std::vector<uint64_t> &all, size_t w, size_t off, int P, size_t mul) {
  uint64_t m = 0;
  for (int q = 0; q < P; ++q)
    for (int r = 0; r < P; ++r) m = std::max<uint64_t>(m, all[(size_t)q * w + off + r]);
  return (size_t)m * mul;
}

// all-to-all of variable segments (words): segment q of send goes to rank q.  gmax = the
// largest segment any rank sends to any rank (every rank passes the same value).
nut_status alltoallv(nut_dist *d, int l, const uint64_t *send, const size_t *sc, const size_t *sd, uint64_t *recv,
                     const size_t *rc, const size_t *rd, size_t gmax) {
  Member &mb = d->m[l];
  hipStream_t s = mb.ctx->stream;
  if (d->mode != nut_dist::kVirtual) {
    const int P = d->nranks;
    const size_t rounds = std::max<size_t>(1, (gmax + kA2AChunk - 1) / kA2AChunk);
    std::vector<size_t> c1(P), d1(P), c2(P), d2(P);
    for (size_t k = 0; k < rounds; ++k) {
      const size_t o = k * kA2AChunk;
      for (int q = 0; q < P; ++q) {
        c1[q] = sc[q] > o ? std::min(kA2AChunk, sc[q] - o) : 0;
        d1[q] = sd[q] + o;
        c2[q] = rc[q] > o ? std::min(kA2AChunk, rc[q] - o) : 0;
        d2[q] = rd[q] + o;
      }
      ncclResult_t e = rounds == 1 ? d->r->all_to_allv(send, sc, sd, recv, rc, rd, ncclUint64, mb.comm, s)
                                   : d->r->all_to_allv(send, c1.data(), d1.data(), recv, c2.data(), d2.data(), ncclUint64,
                                                       mb.comm, s);
      (void)hipGetLastError();
      if (e != ncclSuccess) return rccl_fail(d->r, e, "ncclAllToAllv");
    }
    return NUT_OK;
  }
  Hub &h = d->hub;
  const int me = mb.rank;
  NUT_HIP(hipStreamSynchronize(s));
  h.post[l] = Hub::Post{send, sc, sd, 0};
  h.barrier();
  hipError_t e = hipSuccess;
  nut_status st = NUT_OK;
  for (int q = 0; q < d->nranks && e == hipSuccess; ++q) {
    const Hub::Post &p = h.post[q];
    if (p.count[me] != rc[q]) {
      st = fail(NUT_ERR_INVALID_ARG, "nut_dist (virtual) all-to-all: receive count mismatch");
      break;
    }
    if (rc[q]) e = hipMemcpyAsync(recv + rd[q], p.send + p.displ[me], rc[q] * 8, hipMemcpyDeviceToDevice, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  h.barrier();
  if (st) return st;
  return e == hipSuccess ? NUT_OK : hip_fail(e, "nut_dist (virtual) all-to-all");
}

// Several all-to-alls as one exchange: RCCL runs them inside one ncclGroupStart / End
// (every link carries all of them at once, one launch and one completion), in rounds in
// which no (sender, receiver) pair moves more than kA2AChunk words over all of them
// together (RCCL's per-transfer limit, above).  Virtual ranks run them one after another.
struct A2A {
  const uint64_t *send;
  const size_t *sc, *sd;
  uint64_t *recv;
  const size_t *rc, *rd;
};
nut_status alltoallv_group(nut_dist *d, int l, const std::vector<A2A> &ops, size_t gmax) {
  if (d->mode == nut_dist::kVirtual) {
    for (const A2A &o : ops) {
      nut_status st = alltoallv(d, l, o.send, o.sc, o.sd, o.recv, o.rc, o.rd, gmax);
      if (st) return st;
    }
    return NUT_OK;
  }
  Member &mb = d->m[l];
  hipStream_t s = mb.ctx->stream;
  const int P = d->nranks;
  const size_t chunk = kA2AChunk / std::max<size_t>(ops.size(), 1);
  const size_t rounds = std::max<size_t>(1, (gmax + chunk - 1) / chunk);
  std::vector<size_t> c1(P), d1(P), c2(P), d2(P);
  for (size_t k = 0; k < rounds; ++k) {
    const size_t o = k * chunk;
    ncclResult_t e = d->r->group_start();
    for (size_t i = 0; i < ops.size() && e == ncclSuccess; ++i) {
      const A2A &a = ops[i];
      for (int q = 0; q < P; ++q) {
        c1[q] = a.sc[q] > o ? std::min(chunk, a.sc[q] - o) : 0;
        d1[q] = a.sd[q] + o;
        c2[q] = a.rc[q] > o ? std::min(chunk, a.rc[q] - o) : 0;
        d2[q] = a.rd[q] + o;
      }
      e = d->r->all_to_allv(a.send, c1.data(), d1.data(), a.recv, c2.data(), d2.data(), ncclUint64, mb.comm, s);
    }
    const ncclResult_t e2 = d->r->group_end();
    (void)hipGetLastError();
    if (e != ncclSuccess) return rccl_fail(d->r, e, "ncclAllToAllv (grouped)");
    if (e2 != ncclSuccess) return rccl_fail(d->r, e2, "ncclGroupEnd");
  }
  return NUT_OK;
}

// All-gather of a `w`-word host header whose word 0 is this rank's status.  On return
// all[q * w + i] holds rank q's header; NUT_OK only if every rank reported NUT_OK.
nut_status exchange_header(nut_dist *d, int l, nut_status mine, const std::vector<uint64_t> &hdr,
                           std::vector<uint64_t> &all) {
  Member &mb = d->m[l];
  const size_t w = hdr.size();
  std::string my_error = mine ? nut_last_error() : "";
  uint64_t *dev = (uint64_t *)mb.hdr_dev.ptr;
  hipStream_t s = mb.ctx->stream;
  if (w > kHdrWords) return fail(NUT_ERR_INVALID_ARG, "nut_dist: header too wide");
  // staged in page-locked memory: the copy is stream-ordered, no host wait before the
  // all-gather (the one synchronization is the read-back below)
  memcpy(mb.hdr_send, hdr.data(), w * 8);
  mb.hdr_send[0] = (uint64_t)mine;
  NUT_HIP(hipMemcpyAsync(dev, mb.hdr_send, w * 8, hipMemcpyHostToDevice, s));
  nut_status st = allgather(d, l, dev, dev + w, w);
  if (st) return st;
  NUT_HIP(hipMemcpyAsync(mb.hdr_host, dev + w, w * d->nranks * 8, hipMemcpyDeviceToHost, s));
  NUT_HIP(hipStreamSynchronize(s));
  all.assign(mb.hdr_host, mb.hdr_host + w * d->nranks);
  if (mine) return fail(mine, my_error);
  for (int q = 0; q < d->nranks; ++q)
    if (all[(size_t)q * w])
      return fail((nut_status)all[(size_t)q * w], "nut_dist: rank " + std::to_string(q) + " failed (status " +
                                                      std::to_string(all[(size_t)q * w]) + ")");
  return NUT_OK;
}

nut_status agree(nut_dist *d, int l, nut_status mine) {
  std::vector<uint64_t> all;
  return exchange_header(d, l, mine, std::vector<uint64_t>(1, 0), all);
}

// A rank's receive buffers only grow (Scratch), so in steady state they already hold what
// the next exchange brings and reserving them cannot fail.  Each header carries the rank's
// capacities (words); after the header every rank knows every rank's needs, so all ranks
// take the same decision: `agree` on the reservations only when some rank must grow one
// (a failed hipMalloc then fails the call on every rank instead of leaving the others in
// the all-to-all), else no second all-gather.
uint64_t cap_words(const Member &mb, int i) { return mb.buf[i].bytes / 8; }
bool any_growth(const std::vector<uint64_t> &all, size_t w, size_t cap0, int P, int ncap,
                const std::function<uint64_t(int q, int k)> &need) {
  for (int q = 0; q < P; ++q)
    for (int k = 0; k < ncap; ++k)
      if (std::max<uint64_t>(need(q, k), 1) > all[(size_t)q * w + cap0 + k]) return true;
  return false;
}

// run f(l) for every local member: one host thread per member when there are several
template <class F>
nut_status run_members(nut_dist *d, F &&f) {
  const int L = (int)d->m.size();
  if (L == 1) {
    DeviceGuard dg(d->m[0].ctx->device);
    return f(0);
  }
  std::vector<nut_status> st(L, NUT_OK);
  std::vector<std::string> err(L);
  std::vector<std::thread> th;
  th.reserve(L);
  for (int l = 0; l < L; ++l)
    th.emplace_back([&, l] {
      (void)hipSetDevice(d->m[l].ctx->device);
      (void)hipGetLastError();
      st[l] = f(l);
      if (st[l]) err[l] = nut_last_error();
    });
  for (auto &t : th) t.join();
  // report the first member that failed on its own rather than through another's status
  int pick = -1;
  for (int l = 0; l < L && pick < 0; ++l)
    if (st[l] && err[l].rfind("nut_dist: rank", 0) != 0) pick = l;
  for (int l = 0; l < L && pick < 0; ++l)
    if (st[l]) pick = l;
  return pick < 0 ? NUT_OK : fail(st[pick], err[pick]);
}

nut_status member_init(nut_dist *d, Member &mb, int device) {
  nut_status st = nut_ctx_create(device, &mb.ctx);
  if (st) return st;
  DeviceGuard dg(device);
  st = mb.hdr_dev.reserve(kHdrBytes * 2);
  if (st) return st;
  NUT_HIP(hipHostMalloc((void **)&mb.hdr_host, kHdrBytes, hipHostMallocDefault));
  NUT_HIP(hipHostMalloc((void **)&mb.hdr_send, (kHdrWords + kSamples) * 8, hipHostMallocDefault));
  // the sample sort's positions, own sample and pooled samples: reserved here, so the
  // sample all-gather (which carries the status) never waits on an allocation
  return reserve(mb, 3, kSamples + (uint64_t)(d->nranks + 1) * kSampleWords);
}

void member_free(Member &mb) {
  if (!mb.ctx) return;
  {
    DeviceGuard dg(mb.ctx->device);
    (void)hipStreamSynchronize(mb.ctx->stream);
    for (auto &b : mb.buf) b.release();
    mb.hdr_dev.release();
    if (mb.hdr_host) (void)hipHostFree(mb.hdr_host);
    if (mb.hdr_send) (void)hipHostFree(mb.hdr_send);
    mb.hdr_host = mb.hdr_send = nullptr;
  }
  nut_ctx_destroy(mb.ctx);
  mb.ctx = nullptr;
}

nut_status check_dist(nut_dist *d, const char *what) {
  if (!d || d->m.empty()) return fail(NUT_ERR_INVALID_ARG, std::string(what) + ": NULL nut_dist");
  return NUT_OK;
}

// ------------------------------------------------------------------ group-by
// The owners' merged groups reach rank 0 in one all-to-all with no second header when they
// are few: owner q holds at most bound_q = the partial groups it received (known to every
// rank from the first header), so it sends a fixed 1 + W x bound_q words — its group count
// first, then its groups column-major — and rank 0 reads the counts from the segments.
// Above this many words the padding would cost more than a header: exact counts then.
constexpr uint64_t kPaddedGather = 1ull << 20;

nut_status groupby_member(nut_dist *d, int l, const nut_agg_spec *spec, uint64_t hint, nut_groups **out) {
  Member &mb = d->m[l];
  nut_ctx *c = mb.ctx;
  const int P = d->nranks, me = mb.rank;
  *out = nullptr;
  if (P == 1) return nut_groupby(c, spec, hint, out);  // one rank: its groups are the result
  // 1. local pre-aggregation, partial groups partitioned by owner rank
  nut_groups *g = nullptr;
  uint64_t n = 0;
  int W = 0;
  std::vector<uint64_t> counts(P, 0);
  nut_status st = nut_groupby(c, spec, hint, &g);
  if (!st) st = nut_groups_size(g, &n);
  if (!st) {
    W = groups_width(g);
    st = reserve(mb, 0, (uint64_t)W * n);
  }
  if (!st) st = nut_groups_partition(g, P, buf(mb, 0), n, counts.data());
  // header: [status, W, counts to each rank, capacity of buffers 1 and 2]
  const size_t w = 4 + (size_t)P, cw = 2 + (size_t)P;
  std::vector<uint64_t> hdr(w, 0), all;
  hdr[1] = (uint64_t)W;
  for (int q = 0; q < P; ++q) hdr[2 + q] = counts[q];
  hdr[cw] = cap_words(mb, 1);
  hdr[cw + 1] = cap_words(mb, 2);
  st = exchange_header(d, l, st, hdr, all);
  if (st) {
    nut_groups_free(g);
    return st;
  }
  for (int q = 0; q < P; ++q)
    if (all[(size_t)q * w + 1] != (uint64_t)W) {
      nut_groups_free(g);
      return fail(NUT_ERR_INVALID_ARG, "nut_dist_groupby: ranks passed specs of different shapes");
    }
  auto cnt = [&](int from, int to) { return all[(size_t)from * w + 2 + to]; };
  // bound[q]: the partial groups owner q receives (>= its merged groups)
  std::vector<uint64_t> bound(P, 0);
  for (int q = 0; q < P; ++q)
    for (int p = 0; p < P; ++p) bound[q] += cnt(p, q);
  uint64_t gather_words = 0;
  for (int q = 1; q < P; ++q) gather_words += 1 + (uint64_t)W * bound[q];
  const bool padded = gather_words <= kPaddedGather;
  // buffer 1: the partial groups received, and rank 0's gathered segments; buffer 2: owner
  // q's padded segment (buffer 0 holds the partition until the exchange has sent it)
  auto need = [&](int q, int k) -> uint64_t {
    if (k == 0) return std::max<uint64_t>((uint64_t)W * bound[q], padded && q == 0 ? gather_words : 0);
    return padded && q ? 1 + (uint64_t)W * bound[q] : 0;
  };
  if (any_growth(all, w, cw, P, 2, need)) {
    st = reserve(mb, 1, need(me, 0));
    if (!st) st = reserve(mb, 2, need(me, 1));
    st = agree(d, l, st);
    if (st) {
      nut_groups_free(g);
      return st;
    }
  }
  // 2. all-to-all of the partial groups (column-major segments of W words per group)
  std::vector<size_t> sc(P), sd(P), rc(P), rd(P);
  size_t stot = 0, rtot = 0;
  for (int q = 0; q < P; ++q) {
    sc[q] = (size_t)W * counts[q];
    sd[q] = stot;
    stot += sc[q];
    rc[q] = (size_t)W * cnt(q, me);
    rd[q] = rtot;
    rtot += rc[q];
  }
  size_t gmax = 0;
  for (int p = 0; p < P; ++p)
    for (int q = 0; q < P; ++q) gmax = std::max<size_t>(gmax, (size_t)W * cnt(p, q));
  st = alltoallv(d, l, buf(mb, 0), sc.data(), sd.data(), buf(mb, 1), rc.data(), rd.data(), gmax);
  // 3. the owner merges what it received
  nut_groups *own = nullptr;
  nut_prog_node nodes[NUT_MAX_AGGS];
  nut_agg_spec ms;
  for (int q = 0; q < P && !st; ++q) {
    const uint64_t cq = rc[q] / W;
    if (!cq && (own || q + 1 < P)) continue;
    groups_merge_spec(g, buf(mb, 1) + rd[q], cq, &ms, nodes);  // cq = 0: an empty result of g's shape
    st = own ? nut_groupby_accumulate(c, &ms, own) : nut_groupby(c, &ms, hint, &own);
  }
  nut_groups_free(g);
  // 4. the owners' groups are gathered on rank 0, which folds them into its own
  uint64_t n_own = 0;
  if (!st) st = nut_groups_size(own, &n_own);
  std::vector<uint64_t> n_of(P, 0);  // rank 0: each owner's group count
  std::fill(sc.begin(), sc.end(), 0);
  std::fill(sd.begin(), sd.end(), 0);
  std::fill(rc.begin(), rc.end(), 0);
  if (padded) {
    // fixed segments; a failed owner sends a count of ~0 in its segment (every rank still
    // takes part in the all-to-all), and rank 0 fails the call on reading it
    if (me != 0) {
      uint64_t *seg = buf(mb, 2);
      if (!st && n_own) st = nut_groups_to_device(own, seg + 1, n_own);
      mb.hdr_send[0] = st ? ~0ull : n_own;
      hipError_t e = hipMemcpyAsync(seg, mb.hdr_send, 8, hipMemcpyHostToDevice, c->stream);
      if (e != hipSuccess && !st) st = hip_fail(e, "nut_dist_groupby");
      sc[0] = 1 + (size_t)W * bound[me];
    }
    rtot = 0;
    for (int q = 0; q < P; ++q) {
      rd[q] = rtot;
      if (me == 0 && q != 0) rc[q] = 1 + (size_t)W * bound[q];
      rtot += rc[q];
    }
    size_t pmax = 0;
    for (int q = 1; q < P; ++q) pmax = std::max<size_t>(pmax, 1 + (size_t)W * bound[q]);
    nut_status a2a = alltoallv(d, l, buf(mb, 2), sc.data(), sd.data(), buf(mb, 1), rc.data(), rd.data(), pmax);
    if (!st) st = a2a;
    if (me == 0 && !st) {
      for (int q = 1; q < P && !st; ++q) {
        hipError_t e = hipMemcpyAsync(mb.hdr_host + q, buf(mb, 1) + rd[q], 8, hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) st = hip_fail(e, "nut_dist_groupby");
      }
      hipError_t e = st ? hipSuccess : hipStreamSynchronize(c->stream);
      if (e != hipSuccess) st = hip_fail(e, "nut_dist_groupby");
      for (int q = 1; q < P && !st; ++q) {
        n_of[q] = mb.hdr_host[q];
        if (n_of[q] == ~0ull) st = fail(NUT_ERR_HIP, "nut_dist: rank " + std::to_string(q) + " failed its owner merge");
        else if (n_of[q] > bound[q]) st = fail(NUT_ERR_INVALID_ARG, "nut_dist_groupby: owner group count above its bound");
        rd[q] += 1;  // the groups follow the count word
      }
    }
  } else {
    if (!st && me != 0) st = reserve(mb, 0, (uint64_t)W * n_own);
    if (!st && me != 0) st = nut_groups_to_device(own, buf(mb, 0), n_own);
    std::vector<uint64_t> h2(2, 0);
    h2[1] = n_own;
    st = exchange_header(d, l, st, h2, all);
    if (!st) {
      rtot = 0;
      for (int q = 0; q < P; ++q) {
        rd[q] = rtot;
        n_of[q] = all[(size_t)q * 2 + 1];
        if (me == 0 && q != 0) rc[q] = (size_t)W * n_of[q];
        rtot += rc[q];
      }
      if (me != 0) sc[0] = (size_t)W * n_own;
      st = agree(d, l, reserve(mb, 1, rtot));
    }
    size_t pmax = 0;
    for (int q = 0; q < P && !st; ++q) pmax = std::max<size_t>(pmax, (size_t)W * n_of[q]);
    if (!st) st = alltoallv(d, l, buf(mb, 0), sc.data(), sd.data(), buf(mb, 1), rc.data(), rd.data(), pmax);
  }
  if (!st && me == 0) {
    for (int q = 1; q < P && !st; ++q) {
      if (!n_of[q]) continue;
      groups_merge_spec(own, buf(mb, 1) + rd[q], n_of[q], &ms, nodes);
      st = nut_groupby_accumulate(c, &ms, own);
    }
  }
  if (!st) st = nut_ctx_sync(c);
  if (st || me != 0) {
    nut_groups_free(own);
    return st;
  }
  *out = own;
  return NUT_OK;
}

// ------------------------------------------------------------------ sample sort
// Skew-safe key ranges.  s = the P-1 splitters at the pooled sample's quantiles (ascending,
// repeating when one key fills several quantiles).  A key k goes to rank #{i : s[i] <= k}
// — except a key equal to a splitter value v at positions a..b of s: it may sit on any of
// the ranks a .. b+1 (the ranks between hold only v, so the ranks' outputs still
// concatenate in order).  Such keys get a bucket of their own in the partition (splitters
// v and v+1: [v, v+1) = {v}); every bucket maps to a rank range, and the all-to-all splits
// an equal-key bucket's count over that range in proportion to how much of v's run in the
// sorted pooled sample falls in each rank's quantile range (so a key holding half the rows
// fills the ranks around it instead of doubling one).  All distinct splitter values get
// such a bucket when <= 63 splitters result, otherwise the repeated ones (a key holding
// >= 1/P of the sample) — always <= P - 1 splitters.
struct SortRanges {
  std::vector<int64_t> e;  // partition splitters, strictly ascending (nut_partition_i64)
  std::vector<int> lo, hi; // bucket j (keys in [e[j-1], e[j])) -> ranks lo[j] .. hi[j]
  std::vector<std::vector<uint64_t>> w;  // bucket j's weights over lo[j] .. hi[j] (sum > 0)
};

// pool: the sorted pooled sample (s[i] = pool[(i + 1) * m / P])
SortRanges sort_ranges(const std::vector<int64_t> &s, const std::vector<int64_t> &pool, int P) {
  struct V {
    int64_t v;
    int a, b;
  };
  std::vector<V> vs;
  for (int i = 0; i < (int)s.size(); ++i)
    if (vs.empty() || vs.back().v != s[i]) vs.push_back(V{s[i], i, i});
    else vs.back().b = i;
  auto count_e = [&](bool all) {
    int m = 0;
    for (size_t i = 0; i < vs.size(); ++i) {
      ++m;
      const bool eq = all || vs[i].b > vs[i].a;
      if (eq && vs[i].v != INT64_MAX && !(i + 1 < vs.size() && vs[i + 1].v == vs[i].v + 1)) ++m;
    }
    return m;
  };
  const bool all = count_e(true) <= 63;
  const uint64_t m = pool.size();
  SortRanges r;
  auto one = [&](int rank) {
    r.lo.push_back(rank);
    r.hi.push_back(rank);
    r.w.push_back(std::vector<uint64_t>(1, 1));
  };
  one(0);  // bucket 0: keys below every splitter
  for (size_t i = 0; i < vs.size(); ++i) {
    const V &x = vs[i];
    const bool eq = all || x.b > x.a;
    r.e.push_back(x.v);
    if (eq) {  // bucket {v}: ranks a .. b+1, weighted by v's run [f, l) in the pool
      const uint64_t f = (uint64_t)(std::lower_bound(pool.begin(), pool.end(), x.v) - pool.begin());
      const uint64_t l = (uint64_t)(std::upper_bound(pool.begin(), pool.end(), x.v) - pool.begin());
      std::vector<uint64_t> w;
      uint64_t tot = 0;
      for (int t = x.a; t <= x.b + 1; ++t) {
        const uint64_t q0 = (uint64_t)t * m / P, q1 = (uint64_t)(t + 1) * m / P;
        const uint64_t o = std::min(l, q1) > std::max(f, q0) ? std::min(l, q1) - std::max(f, q0) : 0;
        w.push_back(o);
        tot += o;
      }
      if (!tot) std::fill(w.begin(), w.end(), 1);
      r.lo.push_back(x.a);
      r.hi.push_back(x.b + 1);
      r.w.push_back(std::move(w));
      if (x.v != INT64_MAX && !(i + 1 < vs.size() && vs[i + 1].v == x.v + 1)) {
        r.e.push_back(x.v + 1);  // keys in (v, next splitter value): rank b+1
        one(x.b + 1);
      }
    } else {  // keys in [v, next): rank b+1, as without the tie split
      one(x.b + 1);
    }
  }
  return r;
}

// count c of bucket j split over its ranks by weight (cumulative rounding: sums to c)
void split_bucket(const SortRanges &r, size_t j, uint64_t c, std::vector<uint64_t> &counts) {
  const std::vector<uint64_t> &w = r.w[j];
  uint64_t W = 0, acc = 0, prev = 0;
  for (uint64_t x : w) W += x;
  for (size_t t = 0; t < w.size(); ++t) {
    acc += w[t];
    const uint64_t upto = (uint64_t)((unsigned __int128)c * acc / W);
    counts[r.lo[j] + t] += upto - prev;
    prev = upto;
  }
}

nut_status sort_member(nut_dist *d, int l, const int64_t *in, uint64_t n, const int64_t **out, uint64_t *out_n) {
  Member &mb = d->m[l];
  nut_ctx *c = mb.ctx;
  const int P = d->nranks, me = mb.rank;
  hipStream_t s = c->stream;
  if (P == 1) {  // one rank: no samples, no partition, no exchange — the local sort of the input
    nut_status st = reserve(mb, 2, n);
    if (!st && n) {
      DeviceGuard dg(c->device);
      st = nut::msd_sort_i64(c, in, (int64_t *)buf(mb, 2), n, kSortFlip);
    }
    if (!st) st = nut_ctx_sync(c);
    if (st) return st;
    *out = (const int64_t *)buf(mb, 2);
    *out_n = n;
    return NUT_OK;
  }
  // 1. a strided sample of the local keys, all-gathered with its status and whether the
  //    rank has keys (one all-gather, no header before it); splitters at the pooled quantiles
  nut_status st = NUT_OK;
  uint64_t *smp = buf(mb, 3) + kSamples;  // kSampleWords words (buffer 3: reserved at creation)
  if (n) {
    int64_t *idx = (int64_t *)mb.hdr_send;  // page-locked: the copy needs no host wait
    for (int i = 0; i < kSamples; ++i) idx[i] = (int64_t)(((unsigned __int128)i * n) / kSamples);
    int64_t *didx = (int64_t *)buf(mb, 3);
    hipError_t e = hipMemcpyAsync(didx, idx, kSamples * 8, hipMemcpyHostToDevice, s);
    st = e == hipSuccess ? nut_gather_u64(c, (const uint64_t *)in, didx, kSamples, 0, smp + 2)
                         : hip_fail(e, "nut_dist_sort_i64 sample indices");
  }
  uint64_t *h2 = mb.hdr_send + kSamples;  // page-locked, after the positions
  h2[0] = (uint64_t)st;
  h2[1] = n ? 1 : 0;
  NUT_HIP(hipMemcpyAsync(smp, h2, 16, hipMemcpyHostToDevice, s));
  const std::string mine_err = st ? nut_last_error() : "";
  constexpr uint64_t kSw = kSampleWords;
  uint64_t *pool_dev = smp + kSw;
  st = allgather(d, l, smp, pool_dev, kSw);
  std::vector<uint64_t> pooled((size_t)P * kSw);
  if (!st) {
    hipError_t e = hipMemcpyAsync(pooled.data(), pool_dev, pooled.size() * 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) st = hip_fail(e, "nut_dist_sort_i64 sample copy");
  }
  if (st) return st;
  if (pooled[(size_t)me * kSw]) return fail((nut_status)pooled[(size_t)me * kSw], mine_err);
  for (int q = 0; q < P; ++q)
    if (pooled[(size_t)q * kSw])
      return fail((nut_status)pooled[(size_t)q * kSw], "nut_dist: rank " + std::to_string(q) + " failed (status " +
                                                           std::to_string(pooled[(size_t)q * kSw]) + ")");
  std::vector<uint64_t> hdr, all;
  std::vector<int64_t> pool((size_t)P * kSamples);
  for (int q = 0; q < P; ++q)
    memcpy(&pool[(size_t)q * kSamples], &pooled[(size_t)q * kSw + 2], kSamples * 8);
  std::vector<int64_t> live;
  live.reserve(pool.size());
  for (int q = 0; q < P; ++q)
    if (pooled[(size_t)q * kSw + 1]) live.insert(live.end(), pool.begin() + (size_t)q * kSamples, pool.begin() + (size_t)(q + 1) * kSamples);
  std::sort(live.begin(), live.end());
  std::vector<int64_t> spl(P - 1, 0);
  for (int i = 1; i < P; ++i) spl[i - 1] = live.empty() ? 0 : live[(live.size() * (size_t)i) / P];
  const SortRanges rg = sort_ranges(spl, live, P);
  // 2. partition into the ranges' buckets (bucket order = destination order; unstable:
  //    the receiver sorts, and equal keys split by position are still equal keys)
  const int nb = (int)rg.e.size() + 1;
  std::vector<uint64_t> bcount(nb, 0), counts(P, 0);
  const uint64_t *send = buf(mb, 0);
  if (nb == 1) {  // one rank: every key stays, in place
    bcount[0] = n;
    send = (const uint64_t *)in;
  } else {
    if (!st) st = reserve(mb, 0, n);
    send = buf(mb, 0);
    if (!st) st = nut::partition_i64_ranges(c, in, n, rg.e.data(), nb - 1, (int64_t *)buf(mb, 0), bcount.data());
  }
  for (int j = 0; j < nb; ++j) split_bucket(rg, (size_t)j, bcount[j], counts);
  // header: [status, counts to each rank, capacity of buffers 1 and 2]
  const size_t w = 3 + (size_t)P;
  hdr.assign(w, 0);
  for (int q = 0; q < P; ++q) hdr[1 + q] = counts[q];
  hdr[1 + P] = P == 1 ? ~0ull : cap_words(mb, 1);  // (one rank sorts its input in place of a copy)
  hdr[2 + P] = cap_words(mb, 2);
  st = exchange_header(d, l, st, hdr, all);
  if (st) return st;
  std::vector<size_t> sc(P), sd(P), rc(P), rd(P);
  size_t stot = 0, rtot = 0;
  for (int q = 0; q < P; ++q) {
    sc[q] = counts[q];
    sd[q] = stot;
    stot += sc[q];
    rc[q] = all[(size_t)q * w + 1 + me];
    rd[q] = rtot;
    rtot += rc[q];
  }
  auto need = [&](int q, int) {
    uint64_t r = 0;
    for (int p = 0; p < P; ++p) r += all[(size_t)p * w + 1 + q];
    return r;
  };
  if (any_growth(all, w, 1 + (size_t)P, P, 2, need)) {
    st = P == 1 ? NUT_OK : reserve(mb, 1, rtot);
    if (!st) st = reserve(mb, 2, rtot);
    st = agree(d, l, st);
  }
  // 3. one all-to-all of keys, then the local radix sort of the received range
  const int64_t *sort_in = (const int64_t *)buf(mb, 1);
  if (P == 1)  // one rank: nothing to exchange, the local sort reads the input
    sort_in = in;
  else if (!st)
    st = alltoallv(d, l, send, sc.data(), sd.data(), buf(mb, 1), rc.data(), rd.data(), max_cell(all, w, 1, P, 1));
  // this rank's key range from its buckets' splitters: the local sort's capped layout
  // spreads exactly that range, not the full 64-bit one
  uint64_t bnd[2] = {~0ull, 0};
  for (int j = 0; j < nb; ++j) {
    if (rg.lo[j] > me || rg.hi[j] < me) continue;
    const uint64_t a = j == 0 ? 0 : (uint64_t)rg.e[j - 1] ^ kSortFlip;
    const uint64_t b = j == nb - 1 ? ~0ull : ((uint64_t)rg.e[j] ^ kSortFlip) - 1;
    bnd[0] = std::min(bnd[0], a);
    bnd[1] = std::max(bnd[1], b);
  }
  if (!st && rtot) {
    DeviceGuard dg(c->device);
    st = nut::msd_sort_i64(c, sort_in, (int64_t *)buf(mb, 2), rtot, kSortFlip, bnd[0] <= bnd[1] ? bnd : nullptr);
  }
  if (!st) st = nut_ctx_sync(c);
  if (st) return st;
  *out = (const int64_t *)buf(mb, 2);
  *out_n = rtot;
  return NUT_OK;
}

// ------------------------------------------------------------------ filter
nut_status filter_member(nut_dist *d, int l, const int64_t *col, uint64_t n, int cmp, int64_t k, int64_t *out,
                         uint64_t *out_n, uint64_t *out_offset) {
  Member &mb = d->m[l];
  uint64_t cnt = 0;
  nut_status st = nut_filter_i64(mb.ctx, col, n, cmp, k, out, &cnt);
  if (d->nranks == 1) {  // one rank: its output starts at 0, no counts to exchange
    *out_n = cnt;
    *out_offset = 0;
    return st;
  }
  std::vector<uint64_t> hdr(2, 0), all;
  hdr[1] = cnt;
  st = exchange_header(d, l, st, hdr, all);
  if (st) return st;
  uint64_t off = 0;
  for (int q = 0; q < mb.rank; ++q) off += all[(size_t)q * 2 + 1];
  *out_n = cnt;
  *out_offset = off;
  return NUT_OK;
}

// ------------------------------------------------------------------ hash join
nut_status join_member(nut_dist *d, int l, const int64_t *build, uint64_t nb, int64_t brow0, const int64_t *probe,
                       uint64_t np, int64_t prow0, int type, const int64_t **pout, const int64_t **bout,
                       uint64_t *npairs) {
  Member &mb = d->m[l];
  nut_ctx *c = mb.ctx;
  const int P = d->nranks, me = mb.rank;
  if (P == 1 && brow0 == 0 && prow0 == 0) {
    // one rank whose rows are the global rows: the local join's pairs are the result (no
    // partition, exchange or row-id gathers)
    // one pass into buffers of a pair per probe row (unique build keys), again at the exact
    // size when build keys repeat
    uint64_t cap = std::max<uint64_t>(np, 1), np2 = 0;
    nut_status st = NUT_OK;
    for (int attempt = 0; attempt < 2; ++attempt) {
      st = reserve(mb, 8, cap);
      if (!st) st = reserve(mb, 9, cap);
      if (!st) st = nut_join_i64_into(c, build, nb, probe, np, type, (int64_t *)buf(mb, 8), (int64_t *)buf(mb, 9), cap,
                                      &np2);
      if (st != NUT_ERR_CAPACITY) break;
      cap = np2;
    }
    if (!st) st = nut_ctx_sync(c);
    if (st) return st;
    *pout = (const int64_t *)buf(mb, 8);
    *bout = (const int64_t *)buf(mb, 9);
    *npairs = np2;
    return NUT_OK;
  }
  // buffers: 0/1 build keys/rows by part, 2/3 probe keys/rows by part, 4..7 received, 8/9 pairs
  std::vector<uint64_t> bc(P, 0), pc(P, 0);
  nut_status st = reserve(mb, 0, nb);
  if (!st) st = reserve(mb, 1, nb);
  if (!st) st = reserve(mb, 2, np);
  if (!st) st = reserve(mb, 3, np);
  if (!st) st = nut_hash_partition_i64(c, build, nb, P, brow0, (int64_t *)buf(mb, 0), (int64_t *)buf(mb, 1), bc.data());
  if (!st) st = nut_hash_partition_i64(c, probe, np, P, prow0, (int64_t *)buf(mb, 2), (int64_t *)buf(mb, 3), pc.data());
  // header: [status, build counts, probe counts, capacities of buffers 4..7]
  const size_t w = 5 + 2 * (size_t)P;
  std::vector<uint64_t> hdr(w, 0), all;
  for (int q = 0; q < P; ++q) hdr[1 + q] = bc[q], hdr[1 + P + q] = pc[q];
  for (int k = 0; k < 4; ++k) hdr[1 + 2 * P + k] = cap_words(mb, 4 + k);
  st = exchange_header(d, l, st, hdr, all);
  if (st) return st;
  std::vector<size_t> bsc(P), bsd(P), brc(P), brd(P), psc(P), psd(P), prc(P), prd(P);
  size_t bs = 0, br = 0, ps = 0, pr = 0;
  for (int q = 0; q < P; ++q) {
    bsc[q] = bc[q], bsd[q] = bs, bs += bc[q];
    psc[q] = pc[q], psd[q] = ps, ps += pc[q];
    brc[q] = all[q * w + 1 + me], brd[q] = br, br += brc[q];
    prc[q] = all[q * w + 1 + P + me], prd[q] = pr, pr += prc[q];
  }
  auto need = [&](int q, int k) {  // buffers 4 / 5: build records received, 6 / 7: probe records
    uint64_t r = 0;
    for (int p = 0; p < P; ++p) r += all[(size_t)p * w + 1 + (k < 2 ? 0 : P) + q];
    return r;
  };
  if (any_growth(all, w, 1 + 2 * (size_t)P, P, 4, need)) {
    st = reserve(mb, 4, br);
    if (!st) st = reserve(mb, 5, br);
    if (!st) st = reserve(mb, 6, pr);
    if (!st) st = reserve(mb, 7, pr);
    st = agree(d, l, st);
  }
  const size_t gmax = std::max(max_cell(all, w, 1, P, 1), max_cell(all, w, 1 + (size_t)P, P, 1));
  // the build and probe records (keys and row ids) in one grouped exchange
  if (!st)
    st = alltoallv_group(d, l,
                         {A2A{buf(mb, 0), bsc.data(), bsd.data(), buf(mb, 4), brc.data(), brd.data()},
                          A2A{buf(mb, 1), bsc.data(), bsd.data(), buf(mb, 5), brc.data(), brd.data()},
                          A2A{buf(mb, 2), psc.data(), psd.data(), buf(mb, 6), prc.data(), prd.data()},
                          A2A{buf(mb, 3), psc.data(), psd.data(), buf(mb, 7), prc.data(), prd.data()}},
                         gmax);
  if (st) return st;
  // local join of what this rank owns; local pair indices -> global rows
  nut_join *j = nullptr;
  uint64_t np2 = 0;
  st = nut_join_i64(c, (const int64_t *)buf(mb, 4), br, (const int64_t *)buf(mb, 6), pr, type, &j, &np2);
  if (!st) st = reserve(mb, 0, np2);  // the send buffers are free again: local pair indices
  if (!st) st = reserve(mb, 1, np2);
  if (!st) st = reserve(mb, 8, np2);
  if (!st) st = reserve(mb, 9, np2);
  if (!st) st = nut_join_write(j, (int64_t *)buf(mb, 0), (int64_t *)buf(mb, 1));
  nut_join_free(j);
  if (!st) st = nut_gather_u64(c, buf(mb, 7), (const int64_t *)buf(mb, 0), np2, ~0ull, buf(mb, 8));
  if (!st) st = nut_gather_u64(c, buf(mb, 5), (const int64_t *)buf(mb, 1), np2, ~0ull, buf(mb, 9));
  if (!st) st = nut_ctx_sync(c);
  if (st) return st;
  *pout = (const int64_t *)buf(mb, 8);
  *bout = (const int64_t *)buf(mb, 9);
  *npairs = np2;
  return NUT_OK;
}

}  // namespace

extern "C" {

nut_status nut_dist_unique_id(void *id) {
  if (!id) return fail(NUT_ERR_INVALID_ARG, "nut_dist_unique_id: NULL id");
  const Rccl *r = rccl();
  if (!r) return fail(NUT_ERR_UNSUPPORTED, g_rccl.load_error);
  ncclUniqueId u;
  ncclResult_t e = r->get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
  memcpy(id, &u, NUT_DIST_ID_BYTES);
  return NUT_OK;
}

nut_status nut_dist_create(int ndev, const int *devs, nut_dist **out) {
  if (!out || !devs || ndev < 1 || ndev > kMaxRanks) return fail(NUT_ERR_INVALID_ARG, "nut_dist_create: bad argument");
  *out = nullptr;
  const Rccl *r = rccl();
  if (!r) return fail(NUT_ERR_UNSUPPORTED, g_rccl.load_error);
  nut_dist *d = new nut_dist();
  d->mode = nut_dist::kRcclAll;
  d->nranks = ndev;
  d->r = r;
  d->m.resize(ndev);
  std::vector<ncclComm_t> comms(ndev, nullptr);
  nut_status st = NUT_OK;
  for (int i = 0; i < ndev && !st; ++i) {
    d->m[i].rank = i;
    st = member_init(d, d->m[i], devs[i]);
  }
  if (!st) {
    ncclResult_t e = r->comm_init_all(comms.data(), ndev, devs);
    (void)hipGetLastError();
    if (e != ncclSuccess) st = rccl_fail(r, e, "ncclCommInitAll");
  }
  for (int i = 0; i < ndev; ++i) d->m[i].comm = comms[i];
  if (st) {
    nut_dist_destroy(d);
    return st;
  }
  *out = d;
  return NUT_OK;
}

nut_status nut_dist_create_rank(int nranks, int rank, const void *id, int device, nut_dist **out) {
  if (!out || !id || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
    return fail(NUT_ERR_INVALID_ARG, "nut_dist_create_rank: bad argument");
  *out = nullptr;
  const Rccl *r = rccl();
  if (!r) return fail(NUT_ERR_UNSUPPORTED, g_rccl.load_error);
  nut_dist *d = new nut_dist();
  d->mode = nut_dist::kRcclRank;
  d->nranks = nranks;
  d->first_rank = rank;
  d->r = r;
  d->m.resize(1);
  d->m[0].rank = rank;
  nut_status st = member_init(d, d->m[0], device);
  if (!st) {
    DeviceGuard dg(device);
    ncclUniqueId u;
    memcpy(&u, id, NUT_DIST_ID_BYTES);
    ncclResult_t e = r->comm_init_rank(&d->m[0].comm, nranks, u, rank);
    (void)hipGetLastError();
    if (e != ncclSuccess) {
      d->m[0].comm = nullptr;
      st = rccl_fail(r, e, "ncclCommInitRank");
    }
  }
  if (st) {
    nut_dist_destroy(d);
    return st;
  }
  *out = d;
  return NUT_OK;
}

nut_status nut_dist_create_virtual(int nranks, int device, nut_dist **out) {
  if (!out || nranks < 1 || nranks > kMaxRanks) return fail(NUT_ERR_INVALID_ARG, "nut_dist_create_virtual: bad argument");
  *out = nullptr;
  nut_dist *d = new nut_dist();
  d->mode = nut_dist::kVirtual;
  d->nranks = nranks;
  d->hub.n = nranks;
  d->hub.post.resize(nranks);
  d->m.resize(nranks);
  nut_status st = NUT_OK;
  for (int i = 0; i < nranks && !st; ++i) {
    d->m[i].rank = i;
    st = member_init(d, d->m[i], device);
  }
  if (st) {
    nut_dist_destroy(d);
    return st;
  }
  *out = d;
  return NUT_OK;
}

nut_status nut_dist_info(const nut_dist *d, int *nranks, int *nlocal, int *first_rank) {
  if (!d) return fail(NUT_ERR_INVALID_ARG, "nut_dist_info: NULL nut_dist");
  if (nranks) *nranks = d->nranks;
  if (nlocal) *nlocal = (int)d->m.size();
  if (first_rank) *first_rank = d->first_rank;
  return NUT_OK;
}

nut_ctx *nut_dist_ctx(nut_dist *d, int local) {
  if (!d || local < 0 || local >= (int)d->m.size()) return nullptr;
  return d->m[local].ctx;
}

void nut_dist_destroy(nut_dist *d) {
  if (!d) return;
  for (auto &mb : d->m) {
    if (mb.comm && d->r) {
      DeviceGuard dg(mb.ctx ? mb.ctx->device : 0);
      if (mb.ctx) (void)hipStreamSynchronize(mb.ctx->stream);
      (void)d->r->comm_destroy(mb.comm);
    }
    mb.comm = nullptr;
    member_free(mb);
  }
  delete d;
}

nut_status nut_dist_groupby(nut_dist *d, const nut_agg_spec *specs, uint64_t group_hint, nut_groups **out) {
  nut_status st = check_dist(d, "nut_dist_groupby");
  if (st) return st;
  if (!specs || !out) return fail(NUT_ERR_INVALID_ARG, "nut_dist_groupby: NULL argument");
  return run_members(d, [&](int l) { return groupby_member(d, l, &specs[l], group_hint, &out[l]); });
}

nut_status nut_dist_sort_i64(nut_dist *d, const int64_t *const *in, const uint64_t *n, const int64_t **out,
                             uint64_t *out_n) {
  nut_status st = check_dist(d, "nut_dist_sort_i64");
  if (st) return st;
  if (!in || !n || !out || !out_n) return fail(NUT_ERR_INVALID_ARG, "nut_dist_sort_i64: NULL argument");
  return run_members(d, [&](int l) { return sort_member(d, l, in[l], n[l], &out[l], &out_n[l]); });
}

nut_status nut_dist_filter_i64(nut_dist *d, const int64_t *const *col, const uint64_t *n, int cmp, int64_t k,
                               int64_t *const *out, uint64_t *out_n, uint64_t *out_offset) {
  nut_status st = check_dist(d, "nut_dist_filter_i64");
  if (st) return st;
  if (!col || !n || !out || !out_n || !out_offset) return fail(NUT_ERR_INVALID_ARG, "nut_dist_filter_i64: NULL argument");
  return run_members(d, [&](int l) {
    return filter_member(d, l, col[l], n[l], cmp, k, out[l], &out_n[l], &out_offset[l]);
  });
}

nut_status nut_dist_join_i64(nut_dist *d, const int64_t *const *build, const uint64_t *nbuild, const int64_t *build_row0,
                             const int64_t *const *probe, const uint64_t *nprobe, const int64_t *probe_row0,
                             int join_type, const int64_t **probe_idx, const int64_t **build_idx, uint64_t *npairs) {
  nut_status st = check_dist(d, "nut_dist_join_i64");
  if (st) return st;
  if (!build || !nbuild || !build_row0 || !probe || !nprobe || !probe_row0 || !probe_idx || !build_idx || !npairs)
    return fail(NUT_ERR_INVALID_ARG, "nut_dist_join_i64: NULL argument");
  return run_members(d, [&](int l) {
    return join_member(d, l, build[l], nbuild[l], build_row0[l], probe[l], nprobe[l], probe_row0[l], join_type,
                       &probe_idx[l], &build_idx[l], &npairs[l]);
  });
}

}  // extern "C"
