"""The sort's capped layout over range-restricted keys.

The capped two-level layout (48 B/key, no histogram passes) maps the keys' own range —
the sample's [min, max] with a margin, or a sample-sort rank's splitter range — onto its
2^18 cells, so a column whose keys fill only part of the int64 space, and every rank of
the multi-GPU sample sort (whose received keys fill 1/P of it), keeps that layout instead
of falling back to the exact one (64 B/key).  Checked here at >= 2^26 keys (the layout
starts at 2^25):
- the path: nut_ctx_sort_stats reports the capped layout (48 B/key, two levels) on every
  range-restricted input and on every rank of virtual P = 2 and P = 8 sample sorts;
- the result: sorted, and the same multiset as the input (order-independent hash, oracle.c)
  — bit-exact against np.sort for one case;
- the fall-backs: keys outside the sampled range (an outlier the strided sample misses)
  and a span too narrow for the layout give the same sorted output through the exact one.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = (1 << 26) + 12345
CAPPED = lambda n: (48 * n, 2)  # noqa: E731  (bytes, levels) of the capped layout


def _check_sorted(out, keys_host, orc, desc=False):
    o = out.cpu().numpy()
    assert len(o) == len(keys_host)
    # (no np.diff: int64 differences of extreme keys overflow)
    assert bool(np.all(o[1:] <= o[:-1]) if desc else np.all(o[1:] >= o[:-1])), "not sorted"
    assert orc.multiset_hash(o) == orc.multiset_hash(keys_host), "not a permutation of the input"


@pytest.mark.parametrize("lo,width", [
    (3 << 60, 1 << 61),                      # one eighth of the key space, aligned
    (-(1 << 62) + 12345, 3_000_000_000_007),  # an odd span, negative keys
    (-(1 << 40), (1 << 41) + 1),             # across zero
    (10**15, 1 << 30),                       # 2^30 values: ~4096 per cell
])
@pytest.mark.parametrize("desc", [False, True])
def test_sort_capped_range_restricted(ex, orc, lo, width, desc):
    keys = ex.gen_column(5, 0x77 + width % 1000, N, a=lo, b=width)
    out = ex.sort_i64(keys, descending=desc)
    assert ex.sort_stats() == CAPPED(N)
    _check_sorted(out, keys.cpu().numpy(), orc, desc)


def test_sort_capped_range_vs_numpy(ex):
    keys = ex.gen_column(5, 0x99, N, a=-(1 << 61), b=(1 << 60) + 77)
    out = ex.sort_i64(keys)
    assert ex.sort_stats() == CAPPED(N)
    assert np.array_equal(out.cpu().numpy(), np.sort(keys.cpu().numpy()))


def test_sort_capped_range_outlier_falls_back(ex, orc):
    """Two keys far outside the range at positions the strided sample skips: level 0 of
    the capped layout flags them and the exact layout sorts the input."""
    keys = ex.gen_column(5, 0x42, N, a=1 << 50, b=1 << 52)
    keys[N // 2 + 3] = -(2**63)
    keys[N // 3 + 5] = 2**63 - 1
    out = ex.sort_i64(keys)
    nbytes, _ = ex.sort_stats()
    assert nbytes > 48 * N  # the exact layout ran
    o = out.cpu().numpy()
    assert o[0] == -(2**63) and o[-1] == 2**63 - 1
    _check_sorted(out, keys.cpu().numpy(), orc)


def test_sort_narrow_span_duplicates(ex, orc):
    """2^20 distinct values for 2^26 keys (64 copies each): correct whichever layout runs."""
    keys = ex.gen_column(5, 0x43, N, a=-5, b=1 << 20)
    out = ex.sort_i64(keys)
    _check_sorted(out, keys.cpu().numpy(), orc)


@pytest.mark.parametrize("P", [2, 8])
def test_virtual_sample_sort_ranks_stay_capped(ex, orc, P):
    """Every rank of a P-rank sample sort (2^26 keys per rank) sorts its received key
    range with the capped layout: the splitter range is passed to the local sort."""
    from nutdb_amd.dist import NutDist
    per = 1 << 26
    keys = ex.gen_column(1, 0x5A + P, P * per)
    torch.cuda.synchronize()
    d = NutDist.virtual(P)
    try:
        outs = d.sort_i64([keys[r * per:(r + 1) * per] for r in range(P)])
        stats = [d.sort_stats(l) for l in range(P)]
    finally:
        d.close()
    for r, (o, st) in enumerate(zip(outs, stats)):
        assert o.numel() >= (1 << 25), (r, o.numel())
        assert st == CAPPED(o.numel()), (r, st, o.numel())
        assert bool((o[1:] >= o[:-1]).all()), r
    for a, b in zip(outs, outs[1:]):
        assert int(a[-1]) <= int(b[0])
    got = torch.cat(outs).cpu().numpy()
    assert orc.multiset_hash(got) == orc.multiset_hash(keys.cpu().numpy())
