"""GPU parity of the library's own multi-GPU path (nut_dist_*, include/nutexec.h):
RCCL inside libnutexec.so, and the torch-free C host (tests/c/host_q1.c).

On the one-GPU box the P > 1 exchange logic runs through nut_dist_create_virtual (P ranks
on one device, exchanges as device copies — the same partition / all-to-all / merge code
as the RCCL ranks), and the RCCL transport itself through nut_dist_create over device 0
and nut_dist_create_rank with one rank.  Results are compared with the C oracle on the
concatenation of the shards: keys, counts, MIN/MAX and dyadic sums bit-exact; f64 sums of
non-dyadic values within 1e-12 relative (north_star)."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from helpers import F64_SUM_RTOL

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


def shards(n, P):
    return [(n * r // P, n * (r + 1) // P) for r in range(P)]


@pytest.fixture(scope="module")
def ND():
    from nutdb_amd.dist import NutDist
    return NutDist


def _groupby_queries(cols, P, n, aggs, nkeys=1):
    from nutdb_amd import AggQuery
    qs = []
    for r0, r1 in shards(n, P):
        keys = [dev(c[r0:r1]) for c in cols["keys"][:nkeys]]
        vals = [dev(c[r0:r1]) for c in cols["vals"]]
        qs.append(AggQuery(keys=keys, values=vals, aggs=aggs, rows=r1 - r0))
    return qs


def _cmp(got, want, f64_sum_cols=()):
    gk, gw = got
    wk, ww = want
    assert np.array_equal(gk, wk), (gk[:5], wk[:5])
    for j in range(ww.shape[1]):
        if j in f64_sum_cols:
            a, b = gw[:, j].view(np.float64), ww[:, j].view(np.float64)
            assert np.all(np.abs(a - b) <= F64_SUM_RTOL * np.abs(b)), j
        else:
            assert np.array_equal(gw[:, j], ww[:, j]), j


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("G", [7, 1000, 100_000, 200_000])
def test_virtual_groupby_vs_oracle(ND, orc, P, G):
    from nutdb_amd import Agg
    n = 1_000_003
    key = orc.gen_column(2, 0x51, n, a=G)
    vd = orc.gen_column(3, 0x52, n)               # dyadic: exact sums
    vi = orc.gen_column(5, 0x53, n, a=-1000, b=2001)
    cols = {"keys": [key], "vals": [vd, vi]}
    aggs = [Agg("sum", "col", (0,)), Agg("count"), Agg("min", "col", (0,)), Agg("max", "col", (0,)),
            Agg("sum", "col", (1,)), Agg("min", "col", (1,))]
    d = ND.virtual(P)
    try:
        out = d.groupby(_groupby_queries(cols, P, n, aggs), group_hint=G)
        assert out[0] is not None and all(o is None for o in out[1:])
        got = out[0].to_host_words()
        out[0].free()
    finally:
        d.close()
    want = orc.groupby([key], [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,)), (0, 0, (1,)), (2, 0, (1,))],
                       values=[vd, vi], cap=G)
    _cmp(got, want)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_virtual_q1_two_keys(ND, orc, P):
    """config 4 across P ranks (P = 8: the driver's 8-GPU split): 2 keys, predicate, the
    fused disc_price expression."""
    from nutdb_amd import Agg, AggQuery
    from nutdb_amd.workloads import Q1_COLS, Q1_DATE_K
    n = 2_000_001
    sd, rf, ls, qty, price, disc = [orc.gen(s, n) for s in Q1_COLS]
    qs = []
    for r0, r1 in shards(n, P):
        qs.append(AggQuery(keys=[dev(rf[r0:r1]), dev(ls[r0:r1])],
                           values=[dev(qty[r0:r1]), dev(price[r0:r1]), dev(disc[r0:r1])],
                           aggs=[Agg("sum", "col", (0,)), Agg("sum", "col", (1,)), Agg("sum", "mul_1m", (1, 2)),
                                 Agg("count")], preds=[(dev(sd[r0:r1]), "<=", Q1_DATE_K)]))
    d = ND.virtual(P)
    try:
        out = d.groupby(qs, group_hint=8)
        got = out[0].to_host_words()
    finally:
        d.close()
    want = orc.groupby([rf, ls], [(0, 0, (0,)), (0, 0, (1,)), (0, 4, (1, 2)), (1, 0, ())],
                       values=[qty, price, disc], preds=[(sd, 1, Q1_DATE_K)], cap=64)
    _cmp(got, want, f64_sum_cols=(0, 1, 2))


def test_virtual_groupby_many_aggregates_and_empty_shard(ND, orc):
    """8 aggregates (> the 4 fused value slots: the owner merge runs in expression mode)
    and a rank whose shard is empty."""
    from nutdb_amd import Agg, AggQuery
    n = 300_000
    key = orc.gen_column(2, 0x61, n, a=50)
    v = orc.gen_column(3, 0x62, n)
    P = 3
    cuts = [(0, 0), (0, 100_000), (100_000, n)]
    aggs = [Agg("sum", "col", (0,)), Agg("count"), Agg("min", "col", (0,)), Agg("max", "col", (0,)),
            Agg("sum", "col", (0,)), Agg("count"), Agg("max", "col", (0,)), Agg("min", "col", (0,))]
    qs = [AggQuery(keys=[dev(key[a:b])], values=[dev(v[a:b])], aggs=aggs, rows=b - a) for a, b in cuts]
    d = ND.virtual(P)
    try:
        got = d.groupby(qs, group_hint=64)[0].to_host_words()
    finally:
        d.close()
    want = orc.groupby([key], [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,)), (0, 0, (0,)), (1, 0, ()),
                               (3, 0, (0,)), (2, 0, (0,))], values=[v], cap=64)
    _cmp(got, want)


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_virtual_sample_sort(ND, orc, P):
    n = 3_000_017
    k = orc.gen_column(1, 0x50, n)
    k[::97] = k[5]  # duplicates across splitters
    d = ND.virtual(P)
    try:
        outs = d.sort_i64([dev(k[a:b]) for a, b in shards(n, P)])
        got = [o.cpu().numpy() for o in outs]
    finally:
        d.close()
    assert np.array_equal(np.concatenate(got), np.sort(k))
    for a, b in zip(got, got[1:]):  # rank ranges: every key of rank r <= every key of rank r+1
        if len(a) and len(b):
            assert a[-1] <= b[0]


@pytest.mark.parametrize("P,heavy", [(2, 0.5), (3, 0.5), (5, 0.5), (8, 0.9), (4, 1.0)])
def test_virtual_sample_sort_heavy_key(ND, orc, P, heavy):
    """Skew-safe ranges: a key holding half (or 90 %, or all) of the rows is
    spread over the ranks whose quantile ranges it fills — the output stays globally
    sorted and every rank stays near n / P keys."""
    n = 2_000_003
    k = orc.gen_column(1, 0x50, n)
    rng = np.random.default_rng(P)
    k[rng.random(n) < heavy] = -77
    d = ND.virtual(P)
    try:
        outs = d.sort_i64([dev(k[a:b]) for a, b in shards(n, P)])
        got = [o.cpu().numpy() for o in outs]
    finally:
        d.close()
    assert np.array_equal(np.concatenate(got), np.sort(k))
    sizes = [len(g) for g in got]
    assert max(sizes) <= 1.15 * n / P, sizes


def test_virtual_filter_offsets(ND, orc):
    n = 1_000_003
    col = orc.gen_column(0, 0x2A, n)
    P = 4
    k = int(0.3 * 2**62)
    d = ND.virtual(P)
    try:
        res = d.filter_i64([dev(col[a:b]) for a, b in shards(n, P)], "<", k)
    finally:
        d.close()
    want = orc.filter_i64(col, 0, k)
    pos = 0
    for vals, off in res:
        assert off == pos
        v = vals.cpu().numpy()
        assert np.array_equal(v, want[pos:pos + len(v)])
        pos += len(v)
    assert pos == len(want)


@pytest.mark.parametrize("how", ["inner", "left", "semi", "anti"])
def test_virtual_join(ND, orc, how):
    P = 3
    nb, np_ = 40_000, 150_000
    b = orc.gen_column(5, 0x71, nb, a=0, b=60_000)       # repeated build keys
    p = orc.gen_column(5, 0x72, np_, a=0, b=80_000)
    d = ND.virtual(P)
    try:
        bs, ps = shards(nb, P), shards(np_, P)
        res = d.join_i64([dev(b[x:y]) for x, y in bs], [dev(p[x:y]) for x, y in ps], how,
                         [x for x, _ in bs], [x for x, _ in ps])
    finally:
        d.close()
    gp = np.concatenate([r[0].cpu().numpy() for r in res])
    gb = np.concatenate([r[1].cpu().numpy() for r in res])
    wp, wb = orc.join_i64(b, p, how)
    og, ow = np.lexsort((gb, gp)), np.lexsort((wb, wp))
    assert np.array_equal(gp[og], wp[ow]) and np.array_equal(gb[og], wb[ow])


def test_virtual_mismatched_specs_fail_on_every_rank(ND, orc):
    """A rank whose local step fails (here: a different spec shape) fails the call on
    every rank through the status header instead of leaving them in the all-to-all."""
    from nutdb_amd import Agg, AggQuery, NutError
    n = 10_000
    key = dev(orc.gen_column(2, 0x51, n, a=10))
    v = dev(orc.gen_column(3, 0x52, n))
    q1 = AggQuery(keys=[key], values=[v], aggs=[Agg("sum", "col", (0,))])
    q2 = AggQuery(keys=[key], values=[v], aggs=[Agg("sum", "col", (0,)), Agg("count")])
    d = ND.virtual(2)
    try:
        with pytest.raises(NutError):
            d.groupby([q1, q2], group_hint=16)
        out = d.groupby([q1, q1], group_hint=16)  # the group is usable afterwards
        assert len(out[0]) == 10
    finally:
        d.close()


def test_rccl_single_device(ND, orc):
    """The RCCL transport: ncclCommInitAll over device 0 and ncclCommInitRank with one
    rank (ncclAllGather + ncclAllToAllv on the member's stream)."""
    from nutdb_amd import Agg
    n = 1_000_003
    key = orc.gen_column(2, 0x51, n, a=1000)
    vd = orc.gen_column(3, 0x52, n)
    want = orc.groupby([key], [(0, 0, (0,)), (1, 0, ())], values=[vd], cap=1000)
    ks = orc.gen_column(1, 0x50, n)
    for make in (lambda: ND.create([0]), lambda: ND.create_rank(1, 0, ND.unique_id(), 0)):
        d = make()
        try:
            assert (d.nranks, d.nlocal) == (1, 1)
            out = d.groupby(_groupby_queries({"keys": [key], "vals": [vd]}, 1, n,
                                             [Agg("sum", "col", (0,)), Agg("count")]), group_hint=1000)
            _cmp(out[0].to_host_words(), want)
            out[0].free()
            s = d.sort_i64([dev(ks)])[0].cpu().numpy()
            assert np.array_equal(s, np.sort(ks))
        finally:
            d.close()


def test_c_host_without_torch():
    """tests/c/host_q1.c: hipMalloc + the C ABI alone (Q1, SQL, filter, sort, nut_dist over
    RCCL and virtual ranks), checked against the C oracle, in a process that never maps
    torch or Python (the binary checks its own /proc/self/maps)."""
    exe = ROOT / "tests" / "c" / "bin" / "host_q1"
    assert exe.exists(), "tests/c/build.py did not run"
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_q1 OK" in r.stdout


@pytest.mark.parametrize("mode", ["rank", "virtual"])
def test_rccl_single_rank_large_sort_filter_join(ND, orc, mode):
    """One rank through the library's exchange at bench-like sizes (2e8 keys, 1.6 GB through
    the all-to-all — one ncclAllToAllv of that size returned wrong data on this image, so the
    library moves large exchanges in rounds of <= 2^26 words per pair): the sort's received
    range, the sort statistics (full-range keys take the capped two-level layout: 48 B/key)
    and the join's global pairs."""
    n = 200_000_003
    ks = orc.gen_column(1, 0x50, n)
    d = ND.create_rank(1, 0, ND.unique_id(), 0) if mode == "rank" else ND.virtual(1)
    try:
        s = d.sort_i64([dev(ks)])[0].cpu().numpy()
        nbytes, levels = d.sort_stats()
        assert np.array_equal(s, np.sort(ks))
        assert (nbytes, levels) == (48 * n, 2)
        b = orc.gen_column(0, 0x71, 2_000_000)
        p = np.where(ks[:8_000_000] % 10 == 0, ks[:8_000_000] | (1 << 62), b[ks[:8_000_000] % 2_000_000])
        pi, bi = d.join_i64([dev(b)], [dev(p)], "inner")[0]
        pi, bi = pi.cpu().numpy(), bi.cpu().numpy()
        o = np.lexsort((bi, pi))
        wp, wb = orc.join_i64(b, p, "inner")
        assert np.array_equal(pi[o], wp) and np.array_equal(bi[o], wb)
    finally:
        d.close()


@pytest.mark.parametrize("mode", ["rank", "virtual"])
def test_rccl_join_grouped_exchange_in_rounds(ND, orc, mode):
    """The join's exchange as one grouped exchange (ncclGroupStart / End around the four
    all-to-alls) in more than one round: row offsets keep one rank off the
    P = 1 shortcut, and 3e7 probe records put each of the four transfers over the 2^24-word
    share of a round (RCCL's 2^30-byte per-transfer limit split four ways)."""
    nb, np_ = 4_000_000, 30_000_001
    b = orc.gen_column(0, 0x81, nb)
    sel = orc.gen_column(5, 0x82, np_, a=0, b=nb)
    p = b[sel]
    p[::7] ^= 1 << 62  # ~1/7 of the probe rows match nothing
    d = ND.create_rank(1, 0, ND.unique_id(), 0) if mode == "rank" else ND.virtual(1)
    try:
        pi, bi = d.join_i64([dev(b)], [dev(p)], "inner", [1000], [7])[0]
        pi, bi = pi.cpu().numpy(), bi.cpu().numpy()
    finally:
        d.close()
    wp, wb = orc.join_i64(b, p, "inner")
    o = np.lexsort((bi, pi))
    assert np.array_equal(pi[o], wp + 7) and np.array_equal(bi[o], wb + 1000)
