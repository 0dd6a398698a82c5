"""The copy-floor probe (nut_stream_probe): the bytes it stores are the
read stream's chunks at the stated read:write ratio, and it reports a positive device time.
bench.py divides the same algorithmic bytes by its time to give roofline.copy_floor."""
import ctypes as C

import numpy as np
import pytest
import torch

from nutdb_amd._lib import lib

pytestmark = pytest.mark.gpu


def _probe(ex, src, dst, rb, wb):
    ex._bind_stream()  # the buffers were filled on torch's stream
    ms = C.c_double()
    st = lib.nut_stream_probe(ex.ctx, C.c_void_p(src.data_ptr()), rb, C.c_void_p(dst.data_ptr()), wb, 2, C.byref(ms))
    return st, ms.value


@pytest.mark.parametrize("chunks,q64", [(64 * 37, 32), (64 * 37 + 13, 32), (1000, 64), (4096, 0), (130, 5)])
def test_probe_writes_ratio(ex, chunks, q64):
    rng = np.random.default_rng(chunks + q64)
    src_h = rng.integers(0, 2**63, size=chunks * 2, dtype=np.int64)
    src = torch.from_numpy(src_h).to(ex.device)
    rb = chunks * 16
    wb = rb * q64 // 64 // 16 * 16
    dst = torch.full((wb // 8 + 128,), -1, dtype=torch.int64, device=ex.device)
    st, ms = _probe(ex, src, dst, rb, wb)
    assert st == 0 and ms > 0
    got = dst.cpu().numpy().reshape(-1, 2)
    q = (wb * 64) // rb  # the kernel's own ratio (floor)
    lanes = np.arange(chunks)
    kept = lanes[(lanes & 63) < q]
    want = src_h.reshape(-1, 2)[kept]
    np.testing.assert_array_equal(got[: len(kept)], want)
    assert (got[len(kept):] == -1).all()


def test_probe_rejects_bad_sizes(ex):
    src = torch.zeros(64, dtype=torch.int64, device=ex.device)
    st, _ = _probe(ex, src, src, 100, 0)  # not a multiple of 16
    assert st != 0
    st, _ = _probe(ex, src, src, 256, 512)  # writes more than it reads
    assert st != 0


def test_probe_executor_helper(ex):
    ms = ex.stream_probe(64 << 20, 32 << 20, reps=3)
    assert 0 < ms < 100
