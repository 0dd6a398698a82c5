"""GPU parity of the hash join (csrc/join.hip) and the gather that carries columns through
a join index, against the numpy oracle (oracle/oracle.py join_i64).  Pairs come out in
probe-row order; the build rows of one probe row are in unspecified order, so each probe
row's build rows are compared sorted."""
import numpy as np
import pytest
import torch

from test_gpu_exec import I64_MAX, I64_MIN, dev, host

pytestmark = pytest.mark.gpu

HOW = ["inner", "left", "semi", "anti"]


def canon(pi, bi):
    o = np.lexsort((bi, pi))
    return pi[o], bi[o]


def check(ex, orc, b, p, how):
    pi, bi = ex.join_i64(dev(b, ex), dev(p, ex), how)
    pi, bi = host(pi), host(bi)
    wp, wb = orc.join_i64(b, p, how)
    assert np.all(pi[1:] >= pi[:-1]), "pairs not in probe-row order"
    gp, gb = canon(pi, bi)
    assert np.array_equal(gp, wp) and np.array_equal(gb, wb), how


@pytest.mark.parametrize("how", HOW)
@pytest.mark.parametrize("nb,np_", [(0, 1000), (1000, 0), (1, 1), (100, 5000), (4096, 4097), (100_000, 1_000_003)])
def test_join_unique_build(ex, orc, how, nb, np_):
    rng = np.random.default_rng(nb + np_)
    b = rng.permutation(np.arange(nb, dtype=np.int64) * 7 - 1000)
    p = rng.integers(-2000, 7 * max(nb, 1), np_).astype(np.int64)
    check(ex, orc, b, p, how)


@pytest.mark.parametrize("how", HOW)
def test_join_duplicates_both_sides(ex, orc, how):
    rng = np.random.default_rng(5)
    b = rng.integers(0, 300, 20_000).astype(np.int64)
    p = rng.integers(-50, 350, 30_001).astype(np.int64)
    check(ex, orc, b, p, how)


@pytest.mark.parametrize("how", HOW)
def test_join_extreme_keys(ex, orc, how):
    rng = np.random.default_rng(9)
    pool = np.array([I64_MIN, I64_MAX, 0, -1, 1, 123456789012345], dtype=np.int64)
    b = pool[rng.integers(0, 4, 50)]
    p = pool[rng.integers(0, len(pool), 10_000)]
    check(ex, orc, b, p, how)


def test_join_large_property(ex, orc):
    """1e7 unique build keys, 2e8 probe keys (~90 % matching): count and a checksum of the
    pairs against numpy."""
    nb, np_ = 10_000_000, 200_000_000
    b = ex.gen_column(0, 0x71, nb)  # unique with overwhelming probability (62-bit)
    bh = host(b)
    sel = ex.gen_column(0, 0x72, np_)  # probe: every 10th row misses
    idx = (sel % nb)
    p = torch.where(sel % 10 == 0, sel | (1 << 62), b[idx])
    pi, bi = ex.join_i64(b, p, "inner")
    hp = host(p)
    miss = (host(sel) % 10) == 0
    assert len(pi) == int((~miss).sum())
    assert np.array_equal(host(pi), np.nonzero(~miss)[0])
    assert np.array_equal(bh[host(bi)], hp[~miss])


def test_gather_null_and_f64(ex):
    col = torch.arange(10, dtype=torch.float64, device=ex.device) * 1.5
    idx = torch.tensor([3, -1, 0, 9, -1], dtype=torch.int64, device=ex.device)
    out = host(ex.gather(col, idx, null=-0.25))
    assert out.tolist() == [4.5, -0.25, 0.0, 13.5, -0.25]
    icol = torch.tensor([I64_MIN, 7, I64_MAX], dtype=torch.int64, device=ex.device)
    assert host(ex.gather(icol, torch.tensor([2, 0, -1], device=ex.device), null=-9)).tolist() == [I64_MAX, I64_MIN, -9]
