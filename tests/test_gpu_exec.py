"""GPU parity: the HIP kernels (through the C ABI) vs the C oracle and the golden fixtures.

Bit-exact for integer / index / count / min / max results and for f64 sums of dyadic
values; f64 sums of non-dyadic values within F64_SUM_RTOL = 1e-12 relative
(BASELINE.json north_star).
"""
import numpy as np
import pytest
import torch

from helpers import F64_SUM_RTOL, OPCODE, fromhex, pos_hash, rel_err, wsum

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max


def dev(x, ex):
    return torch.from_numpy(np.ascontiguousarray(x)).to(ex.device)


def host(t):
    return t.cpu().numpy()


# ----------------------------------------------------------------------------- generator
def test_generator(golden, ex):
    for case in golden["generator"]:
        v = host(ex.gen_column(case["kind"], case["seed"], case["n"], row0=case["row0"], a=case["a"],
                               b=case["b"], c=case["c"]))
        assert [int(x) for x in v[:8].view(np.uint64)] == case["head"]
        assert wsum(v) == case["wsum"]


# ----------------------------------------------------------------------------- filter
def test_filter_golden(golden, ex):
    n = golden["filter"][0]["n"]
    col = ex.gen_column(0, 0x2A, n)
    for case in golden["filter"]:
        out = host(ex.filter_i64(col, case["op"], case["k"]))
        assert len(out) == case["count"], case
        assert [int(x) for x in out[:8]] == case["head"]
        assert [int(x) for x in out[-8:]] == case["tail"]
        assert pos_hash(out) == case["pos_hash"]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 511, 4095, 4096, 4097, 8191, 65536 + 3, 1_000_003])
def test_filter_sizes_vs_oracle(ex, orc, n):
    col = orc.gen_column(0, 0x2A, n)
    d = dev(col, ex)
    for s in (0.0, 0.3, 1.0):
        k = int(s * 2**62)
        for op in ("<", ">="):
            got = host(ex.filter_i64(d, op, k))
            want = orc.filter_i64(col, OPCODE[op], k)
            assert np.array_equal(got, want), (n, s, op)


@pytest.mark.parametrize("n", [32767, 32768, 32769, 3 * 32768 - 1, 257 * 32768 + 5])
def test_filter_staged_tiles_vs_oracle(ex, orc, n):
    """The persistent LDS-staged kernel (32768-row tiles, 20224-row buffer): tile-multiple
    and ragged sizes, tiles denser than the buffer (s = 0.62 .. 1, staged in two halves),
    and an output pointer 8 bytes off 16-B alignment (scalar head / tail stores)."""
    col = orc.gen_column(0, 0x2A, n)
    d = dev(col, ex)
    for s in (0.05, 0.5, 0.62, 0.7, 0.95, 1.0):
        k = int(s * 2**62)
        got = host(ex.filter_i64(d, "<", k))
        assert np.array_equal(got, orc.filter_i64(col, OPCODE["<"], k)), (n, s)
    buf = torch.empty(n + 1, dtype=torch.int64, device=ex.device)
    k = int(0.7 * 2**62)
    got = host(ex.filter_i64(d, "<", k, out=buf[1:]))
    assert np.array_equal(got, orc.filter_i64(col, OPCODE["<"], k))


def test_filter_extremes_and_unaligned(ex, orc):
    rng = np.random.default_rng(7)
    v = rng.integers(I64_MIN, I64_MAX, size=50_001, dtype=np.int64)
    v[::97] = I64_MIN
    v[::89] = I64_MAX
    v[::5] = 42
    d = dev(v, ex)
    for op in OPCODE:
        for k in (I64_MIN, -1, 0, 42, I64_MAX):
            assert np.array_equal(host(ex.filter_i64(d, op, k)), orc.filter_i64(v, OPCODE[op], k)), (op, k)
    # 8-byte aligned but not 16-byte aligned column (slice) takes the scalar-load path
    got = host(ex.filter_i64(d[1:], "==", 42))
    assert np.array_equal(got, orc.filter_i64(v[1:], OPCODE["=="], 42))


def test_filter_large_property(ex, orc):
    n = 100_000_000  # BASELINE config 2 size
    col = ex.gen_column(0, 0x2A, n)
    k = int(0.5 * 2**62)
    out = ex.filter_i64(col, "<", k)
    ref = orc.filter_i64(orc.gen_column(0, 0x2A, n), OPCODE["<"], k)
    assert out.numel() == len(ref)
    o = host(out)
    assert np.array_equal(o, ref)


# ----------------------------------------------------------------------------- group-by
def gb_query(key, val, preds=()):
    from nutdb_amd import Agg, AggQuery
    return AggQuery(keys=[key], values=[val], preds=list(preds),
                    aggs=[Agg("sum", "col", (0,)), Agg("count"), Agg("min", "col", (0,)), Agg("max", "col", (0,))])


@pytest.mark.parametrize("idx", range(5))
def test_groupby_golden(golden, ex, idx):
    case = golden["groupby"][idx]
    n, G = case["n"], case["G"]
    key = ex.gen_column(2, 0x51, n, a=G)
    val = ex.gen_column(3 if case["dyadic"] else 4, 0x52, n)
    preds = [(val, "<", case["pred_val_lt"])] if case["pred_val_lt"] is not None else []
    g = ex.groupby(gb_query(key, val, preds), group_hint=G)
    keys, words = g.to_host_words()
    assert [int(k) for k in keys[:, 0]] == case["keys"]
    s = words[:, 0].view(np.float64)
    fs = fromhex(case["sum_fsum"])
    if case["dyadic"]:
        assert np.array_equal(s, fs)
    assert rel_err(s, fs) <= F64_SUM_RTOL
    assert [int(x) for x in words[:, 1]] == case["count"]
    assert np.array_equal(words[:, 2].view(np.float64), fromhex(case["min"]))
    assert np.array_equal(words[:, 3].view(np.float64), fromhex(case["max"]))


def check_vs_oracle(g, okeys, owords, types):
    keys, words = g.to_host_words()
    assert np.array_equal(keys, okeys)
    for j, t in enumerate(types):
        if t == "sum_f64":
            assert rel_err(words[:, j].view(np.float64), owords[:, j].view(np.float64)) <= F64_SUM_RTOL
        else:
            assert np.array_equal(words[:, j], owords[:, j]), t


AGGS4 = [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,))]


@pytest.mark.parametrize("G,hint", [(1, 1), (16, 0), (1000, 1000), (1000, 0), (100_000, 100_000),
                                    (100_000, 1000), (2_000_000, 2_000_000)])
def test_groupby_cardinalities(ex, orc, G, hint):
    n = 3_000_017
    key = orc.gen_column(2, 0x51, n, a=G)
    val = orc.gen_column(4, 0x52, n)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=hint)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    assert len(g) == len(ok)
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


def test_groupby_sentinel_and_extreme_keys(ex, orc):
    rng = np.random.default_rng(3)
    n = 200_000
    pool = np.array([I64_MIN, I64_MAX, 0, -1, 1, 12345], dtype=np.int64)
    key = pool[rng.integers(0, len(pool), n)]
    val = rng.standard_normal(n)
    val[::1000] = -0.0
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=8)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


def test_groupby_i64_values_wrap(ex, orc):
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(5)
    n = 500_003
    key = rng.integers(0, 37, n).astype(np.int64)
    v = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    q = AggQuery(keys=[dev(key, ex)], values=[dev(v, ex)],
                 aggs=[Agg("sum", "col", (0,)), Agg("min", "col", (0,)), Agg("max", "col", (0,)), Agg("count")])
    g = ex.groupby(q, group_hint=37)
    ok, ow = orc.groupby([key], [(0, 0, (0,)), (2, 0, (0,)), (3, 0, (0,)), (1, 0, ())], values=[v])
    check_vs_oracle(g, ok, ow, ["i", "i", "i", "i"])


def test_groupby_two_keys_preds_exprs(ex, orc):
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(11)
    n = 1_000_001
    k1 = rng.integers(-3, 40, n).astype(np.int64)
    k2 = rng.integers(0, 7, n).astype(np.int64) * 1_000_000_007
    a = rng.random(n)
    b = rng.random(n)
    c = rng.random(n)
    f = rng.integers(0, 100, n).astype(np.int64)
    q = AggQuery(keys=[dev(k1, ex), dev(k2, ex)], values=[dev(a, ex), dev(b, ex), dev(c, ex)],
                 preds=[(dev(f, ex), ">=", 10), (dev(a, ex), "<", 0.9)],
                 aggs=[Agg("sum", "mul", (0, 1)), Agg("sum", "mul_1m_1p", (0, 1, 2)), Agg("min", "sub", (1, 2)),
                       Agg("max", "add", (0, 2)), Agg("count"), Agg("sum", "mul_1m", (2, 0))])
    g = ex.groupby(q, group_hint=300)
    ok, ow = orc.groupby([k1, k2], [(0, 1, (0, 1)), (0, 5, (0, 1, 2)), (2, 3, (1, 2)), (3, 2, (0, 2)), (1, 0, ()),
                                    (0, 4, (2, 0))],
                         values=[a, b, c], preds=[(f, OPCODE[">="], 10), (a, OPCODE["<"], 0.9)])
    check_vs_oracle(g, ok, ow, ["sum_f64", "sum_f64", "i", "i", "i", "sum_f64"])


@pytest.mark.parametrize("nk,lo,hi,hint", [(1, 0, 6, 6), (1, -3, 300, 8), (1, 250, 262, 8), (2, 0, 3, 6),
                                           (2, -2, 20, 8), (2, 0, 16, 4), (2, 14, 18, 8)])
def test_groupby_private_direct_map(ex, orc, nk, lo, hi, hint):
    """Private-accumulator kernels (group_hint <= 8): keys inside the direct map's range
    (one key < 256, two keys < 16 each) take their private id from it, keys outside it,
    negative keys and groups beyond the hint go through the hash table — all mixed in
    one launch; bit-exact integer aggregates, f64 sums to 1e-12."""
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(nk * 1000 + lo + hi)
    n = 1_500_007
    keys = [rng.integers(lo, hi, n).astype(np.int64) for _ in range(nk)]
    v = rng.random(n)
    q = AggQuery(keys=[dev(k, ex) for k in keys], values=[dev(v, ex)],
                 aggs=[Agg("sum", "col", (0,)), Agg("count"), Agg("min", "col", (0,)), Agg("max", "col", (0,))])
    g = ex.groupby(q, group_hint=hint)
    ok, ow = orc.groupby(keys, AGGS4, values=[v])
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


def test_groupby_empty_and_tiny(ex, orc):
    for n in (0, 1, 2, 3):
        key = np.arange(n, dtype=np.int64) % 2
        val = np.arange(n, dtype=np.float64)
        g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)))
        if n == 0:
            assert len(g) == 0
            continue
        ok, ow = orc.groupby([key], AGGS4, values=[val])
        check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])
    # predicate that rejects everything
    key = np.arange(1000, dtype=np.int64)
    val = np.ones(1000)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex), [(dev(key, ex), "<", -5)]))
    assert len(g) == 0


def test_groupby_accumulate_and_partition(ex, orc):
    """N virtual ranks on one GPU: local partials -> owner partition -> per-owner merge."""
    from nutdb_amd import Agg, AggQuery
    G, n, P = 5000, 2_000_003, 4
    key = orc.gen_column(2, 0x51, n, a=G)
    val = orc.gen_column(4, 0x52, n)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    shards = np.array_split(np.arange(n), P)
    owners = [None] * P
    for r in range(P):  # rank r's local pre-aggregation, partitioned by owner
        sl = shards[r]
        g = ex.groupby(gb_query(dev(key[sl], ex), dev(val[sl], ex)), group_hint=G)
        buf, counts = g.partition(P)
        w = 1 + 4
        off = 0
        for p in range(P):
            seg = buf[w * off: w * (off + counts[p])].view(w, counts[p]) if counts[p] else None
            off += counts[p]
            if seg is None:
                continue
            kcol = seg[0].contiguous()
            sums = seg[1].contiguous().view(torch.float64)
            cnts = seg[2].contiguous()
            mins = seg[3].contiguous().view(torch.float64)
            maxs = seg[4].contiguous().view(torch.float64)
            q = AggQuery(keys=[kcol], values=[sums, cnts, mins, maxs],
                         aggs=[Agg("sum", "col", (0,)), Agg("sum", "col", (1,)), Agg("min", "col", (2,)),
                               Agg("max", "col", (3,))])
            if owners[p] is None:
                owners[p] = ex.groupby(q, group_hint=G)
            else:
                ex.accumulate(q, owners[p])
    parts = [o.to_host_words() for o in owners if o is not None]
    keys = np.concatenate([p[0] for p in parts])
    words = np.concatenate([p[1] for p in parts])
    order = np.argsort(keys[:, 0], kind="stable")
    keys, words = keys[order], words[order]
    assert np.array_equal(keys, ok)
    assert rel_err(words[:, 0].view(np.float64), ow[:, 0].view(np.float64)) <= F64_SUM_RTOL
    assert np.array_equal(words[:, 1:], ow[:, 1:])


# ----------------------------------------------------------------------------- Q1
@pytest.mark.parametrize("idx", range(2))
def test_q1_golden(golden, ex, idx):
    from nutdb_amd.workloads import Q1_COLS, Q1_DATE_K, gen
    case = golden["q1"][idx]
    cols = [gen(ex, spec, case["n"], row0=case["row0"]) for spec in Q1_COLS]
    g = ex.q1(*cols, date_k=Q1_DATE_K)
    keys, words = g.to_host_words()
    assert len(keys) == len(case["groups"])
    for k, w, ref in zip(keys, words, case["groups"]):
        assert (int(k[0]), int(k[1])) == (ref["returnflag"], ref["linestatus"])
        assert int(w[3]) == ref["count"]
        for j, name in enumerate(["sum_qty", "sum_price", "sum_disc_price"]):
            assert rel_err([w[j:j + 1].view(np.float64)[0]], [float.fromhex(ref[name])]) <= F64_SUM_RTOL


def test_q1_vs_oracle_large(ex, orc):
    from nutdb_amd.workloads import Q1_COLS, Q1_DATE_K, gen
    n = 20_000_011
    cols_d = [gen(ex, spec, n) for spec in Q1_COLS]
    g = ex.q1(*cols_d, date_k=Q1_DATE_K)
    sd, rf, ls, qty, price, disc = [orc.gen(spec, n) for spec in Q1_COLS]
    ok, ow = orc.groupby([rf, ls], [(0, 0, (0,)), (0, 0, (1,)), (0, 4, (1, 2)), (1, 0, ())],
                         values=[qty, price, disc], preds=[(sd, OPCODE["<="], Q1_DATE_K)])
    check_vs_oracle(g, ok, ow, ["sum_f64", "sum_f64", "sum_f64", "i"])


def test_partition_owner_matches_host_hash(ex, orc):
    """Device owner partition (nut_groups_partition) == nutdb_amd.dist.owner_of, for one
    and two keys: the CPU gloo exchange test and the GPU path route identically."""
    from nutdb_amd import Agg, AggQuery
    from nutdb_amd.dist import owner_of
    rng = np.random.default_rng(2)
    n = 300_000
    k1 = rng.integers(I64_MIN, I64_MAX, 5000, dtype=np.int64)[rng.integers(0, 5000, n)]
    k2 = rng.integers(-5, 5, n).astype(np.int64)
    v = rng.random(n)
    for keys in ([k1], [k1, k2]):
        q = AggQuery(keys=[dev(k, ex) for k in keys], values=[dev(v, ex)], aggs=[Agg("count")])
        g = ex.groupby(q, group_hint=6000)
        for P in (2, 3, 8):
            buf, counts = g.partition(P)
            b = host(buf)
            w = len(keys) + 1
            off = 0
            for p in range(P):
                seg = b[w * off: w * (off + counts[p])].reshape(w, counts[p])
                off += counts[p]
                own = owner_of(seg[0], seg[1] if len(keys) == 2 else None, P)
                assert np.all(own == p)
            assert sum(counts) == len(g)


# ----------------------------------------------------------------------------- sort
def test_sort_golden(golden, ex):
    case = golden["sort"][0]
    keys = ex.gen_column(1, 0x50, case["n"])
    out = host(ex.sort_i64(keys))
    assert [int(x) for x in out[:8]] == case["head"]
    assert [int(x) for x in out[-8:]] == case["tail"]
    assert pos_hash(out) == case["pos_hash"]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 63, 64, 65, 2048, 2049, 4095, 4096, 4097, 5119, 5120, 5121, 6144, 6145,
                               8192, 8193, 12289, 24576, 24577, 32767, 32768, 32769, 65537, 1_000_003, 9_000_011])
def test_sort_sizes_vs_oracle(ex, orc, n):
    """Every local-sort class edge (msd_sort.hip ls_class: S <= 2048, M <= 5120 as 512 x 10,
    M2 <= 6144, L <= 24576 keys in one segment) and the multi-level sizes above them."""
    col = orc.gen_column(1, 0x50, n)
    got = host(ex.sort_i64(dev(col, ex)))
    assert np.array_equal(got, orc.sort_i64(col))


@pytest.mark.parametrize("n", [300_007, 3_000_017])
@pytest.mark.parametrize("kind", ["dups", "const", "small_range", "extremes", "negative", "unaligned",
                                  "skewed", "sparse_digits", "top_and_bottom"])
def test_sort_distributions(ex, orc, kind, n):
    """Distributions that drive the MSD sort (msd_sort.hip) through every branch: segments
    of equal keys larger than a local sort (copied), digits constant inside a segment but
    not globally (pass-through levels), varying digits that are not adjacent."""
    rng = np.random.default_rng(9)
    if kind == "dups":
        v = rng.integers(-50, 50, n).astype(np.int64)
    elif kind == "const":
        v = np.full(n, -7, dtype=np.int64)
    elif kind == "small_range":
        v = rng.integers(0, 1 << 20, n).astype(np.int64)      # 5 of 8 digit passes trivial
    elif kind == "extremes":
        v = rng.choice(np.array([I64_MIN, I64_MAX, 0, -1, 1], dtype=np.int64), n)
    elif kind == "negative":
        v = -rng.integers(0, I64_MAX, n, dtype=np.int64)
    elif kind == "skewed":  # half the keys one value, the rest full-range
        v = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
        v[rng.random(n) < 0.5] = 42
    elif kind == "sparse_digits":  # digits 7, 6 take 4 values each, digits 5..2 constant
        v = ((rng.integers(0, 4, n) << 56) | (rng.integers(0, 4, n) << 48) | (0x5A << 24)
             | rng.integers(0, 1 << 16, n)).astype(np.int64)
    elif kind == "top_and_bottom":  # only digits 7 and 0 vary
        v = ((rng.integers(0, 256, n).astype(np.uint64) << np.uint64(56))
             | rng.integers(0, 256, n).astype(np.uint64)).view(np.int64)
    else:
        v = rng.integers(I64_MIN, I64_MAX, n + 1, dtype=np.int64)
    d = dev(v, ex)
    src = d[1:] if kind == "unaligned" else d
    want = orc.sort_i64(v[1:] if kind == "unaligned" else v)
    assert np.array_equal(host(ex.sort_i64(src)), want)


def test_sort_large_property(ex, orc):
    n = 200_000_000
    keys = ex.gen_column(1, 0x50, n)
    out = ex.sort_i64(keys)
    o = host(out)
    assert np.all(o[1:] >= o[:-1])
    assert orc.multiset_hash(o) == orc.multiset_hash(orc.gen_column(1, 0x50, n))


# ----------------------------------------------------------------------------- partition / sample sort
@pytest.mark.parametrize("nsplit", [0, 1, 7, 63])
def test_partition_i64(ex, nsplit):
    rng = np.random.default_rng(nsplit)
    n = 1_000_003
    keys = rng.integers(-50, 50, n, dtype=np.int64) if nsplit == 7 else rng.integers(I64_MIN, I64_MAX, n,
                                                                                        dtype=np.int64)
    keys[:3] = [I64_MIN, I64_MAX, 0]
    spl = np.sort(rng.choice(keys, nsplit, replace=False)) if nsplit else np.zeros(0, np.int64)
    if nsplit == 7:
        spl = np.array([-40, -10, -10, 0, 5, 5, 49], dtype=np.int64)  # repeated splitters: empty buckets
    got, counts = ex.partition_i64(dev(keys, ex), spl)
    b = np.searchsorted(spl, keys, side="right")
    want = keys[np.argsort(b, kind="stable")]
    assert counts == [int(c) for c in np.bincount(b, minlength=nsplit + 1)]
    assert np.array_equal(host(got), want)


def test_sample_sort_virtual_ranks(ex, orc):
    """The multi-GPU sample sort's data path with P virtual ranks on one GPU: every shard
    is partitioned on the device by the same splitters, bucket p of every shard goes to
    'rank' p, each rank radix-sorts what it received; the concatenation is the sort."""
    from nutdb_amd.workloads import SORT_COL
    P, n = 5, 2_000_000
    keys = orc.gen(SORT_COL, n)
    shards = np.array_split(keys, P)
    sample = np.sort(np.concatenate([s[(np.arange(256) * len(s)) // 256] for s in shards]))
    spl = np.array([sample[(i * len(sample)) // P] for i in range(1, P)], dtype=np.int64)
    received = [[] for _ in range(P)]
    for s in shards:
        part, counts = ex.partition_i64(dev(s, ex), spl)
        off = 0
        for p, c in enumerate(counts):
            received[p].append(part[off:off + c])
            off += c
    out = [host(ex.sort_i64(torch.cat(r))) for r in received]
    assert np.array_equal(np.concatenate(out), orc.sort_i64(keys))
    assert all(o[-1] <= out[i + 1][0] for i, o in enumerate(out[:-1]) if len(o) and len(out[i + 1]))


@pytest.mark.parametrize("P", [1, 2, 3, 8, 256])
def test_hash_partition_i64(ex, P):
    """nut_hash_partition_i64 against the host owner function: every part holds exactly the
    rows whose key maps to it (keys with their row ids), parts in order."""
    from nutdb_amd.dist import join_owner
    rng = np.random.default_rng(P)
    n = 700_001
    keys = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    keys[:4] = [I64_MIN, I64_MAX, 0, -1]
    k, r, counts = ex.hash_partition_i64(dev(keys, ex), 1000, P)
    k, r = host(k), host(r)
    own = join_owner(keys, P)
    assert counts == [int(c) for c in np.bincount(own, minlength=P)]
    assert np.array_equal(np.sort(r), np.arange(n) + 1000)
    assert np.array_equal(keys[r - 1000], k)
    off = 0
    for p, c in enumerate(counts):
        assert np.all(own[r[off:off + c] - 1000] == p)
        off += c


def test_join_virtual_ranks(ex, orc):
    """The multi-GPU join's data path with P virtual ranks on one GPU: both sides' shards
    hash-partitioned on the device, part p of every shard joined on 'rank' p; the union of
    the per-rank pairs (global rows) is the single-GPU join."""
    P = 4
    rng = np.random.default_rng(8)
    b = rng.integers(0, 400_000, 500_000).astype(np.int64)
    p = rng.integers(-1000, 500_000, 2_000_003).astype(np.int64)
    recv = [[[], [], [], []] for _ in range(P)]  # per rank: build keys, build rows, probe keys, probe rows
    for side, arr in ((0, b), (2, p)):
        off = 0
        for s in np.array_split(arr, P):
            k, r, counts = ex.hash_partition_i64(dev(s, ex), off, P)
            o = 0
            for q, c in enumerate(counts):
                recv[q][side].append(k[o:o + c])
                recv[q][side + 1].append(r[o:o + c])
                o += c
            off += len(s)
    for how in ("inner", "left", "anti"):
        gps, gbs = [], []
        for q in range(P):
            bk, br, pk, pr = (torch.cat(x) for x in recv[q])
            pi, bi = ex.join_i64(bk, pk, how)
            gps.append(host(pr[pi]))
            gbs.append(np.where(host(bi) >= 0, host(br)[np.maximum(host(bi), 0)], -1))
        gp, gb = np.concatenate(gps), np.concatenate(gbs)
        o = np.lexsort((gb, gp))
        wp, wb = orc.join_i64(b, p, how)
        assert np.array_equal(gp[o], wp) and np.array_equal(gb[o], wb), how


@pytest.mark.parametrize("n", [40_000, 5_000_003])
def test_sort_desc_msd(ex, orc, n):
    """Descending MSD sort: duplicates, extremes and a block of equal keys."""
    rng = np.random.default_rng(11)
    v = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    v[: n // 3] = rng.integers(-3, 3, n // 3)
    v[-4:] = [I64_MIN, I64_MAX, 0, -1]
    out = host(ex.sort_i64(dev(v, ex), descending=True))
    assert np.array_equal(out, np.sort(v)[::-1])


def test_sort_stats(ex):
    """Algorithmic bytes reported for the roofline: full-range keys above one local sort
    take two histogram reads, two scatter levels and the local sort (64 B/key)."""
    n = 20_000_000
    keys = ex.gen_column(1, 0x50, n)
    ex.sort_i64(keys)
    nbytes, levels = ex.sort_stats()
    assert levels == 2 and nbytes == 64 * n


@pytest.mark.parametrize("kind", ["cluster", "narrow_range", "rank_range", "two_clusters_dups"])
def test_sort_deep_levels(ex, orc, kind):
    """MSD levels beyond the second: sub-segments too large for a local
    sort after a device-planned level go back to the host for another level; a narrow key
    range rebases the digits on the minimum (a sample-sort rank's range)."""
    rng = np.random.default_rng(21)
    n = 60_000_000
    if kind == "cluster":          # half the keys inside a 2^40-wide range: 4 levels there
        v = np.concatenate([rng.integers(I64_MIN, I64_MAX, n // 2, dtype=np.int64),
                            (1 << 50) + rng.integers(0, 1 << 40, n - n // 2, dtype=np.int64)])
    elif kind == "narrow_range":   # every key in [x, x + 2^35): rebased digits
        v = (-(1 << 61)) + rng.integers(0, 1 << 35, n, dtype=np.int64)
    elif kind == "rank_range":     # 1/8 of the key space, not aligned to a digit boundary
        lo = I64_MIN // 8 * 3 + 12345
        v = lo + rng.integers(0, 1 << 61, n, dtype=np.int64)
    else:                          # two tight clusters with many duplicates
        v = np.concatenate([rng.integers(0, 1000, n // 2, dtype=np.int64) * (1 << 20),
                            rng.integers(-(1 << 24), -(1 << 24) + 50_000, n - n // 2, dtype=np.int64)])
    rng.shuffle(v)
    o = host(ex.sort_i64(dev(v, ex)))
    assert np.all(o[1:] >= o[:-1])
    assert orc.multiset_hash(o) == orc.multiset_hash(v)
    if kind != "cluster":
        assert np.array_equal(o, np.sort(v))


@pytest.mark.parametrize("n,desc", [(1 << 25, False), (40_000_003, False), (40_000_003, True)])
def test_sort_capped_layout(ex, orc, n, desc):
    """Large full-range inputs take the capped two-level layout (no histogram pass: both
    scatter levels write into regions of ~1.1x their even share, the local sorts place each
    run by a scan of the level-1 cursors): 48 B/key, bit-exact."""
    col = orc.gen_column(1, 0x57, n)
    got = host(ex.sort_i64(dev(col, ex), descending=desc))
    nbytes, levels = ex.sort_stats()
    assert (nbytes, levels) == (48 * n, 2)
    want = orc.sort_i64(col)
    assert np.array_equal(got, want[::-1] if desc else want)


@pytest.mark.parametrize("kind", ["unsampled_skew", "second_digit_skew", "narrow"])
def test_sort_capped_fallback(ex, orc, kind):
    """Inputs the capped layout cannot hold fall back to the exact layout and still sort
    bit-exact: a skew the admission sample does not see (every sampled key random, every
    other key one value) overflows a level-0 region at run time; a second digit that takes
    few values is refused by the sample.  A narrow range is NOT a fallback any more (round
    4): the layout maps the sampled range onto its cells, so it stays capped."""
    n = 1 << 25
    rng = np.random.default_rng(5)
    v = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    if kind == "unsampled_skew":
        keep = np.zeros(n, dtype=bool)
        keep[(np.arange(16384, dtype=np.int64) * n) // 16384] = True
        v[~keep] = 77
    elif kind == "second_digit_skew":
        v = (v & ~np.int64(0x7FC00000000000)) | (np.int64(3) << 46)
    else:
        v = rng.integers(0, 1 << 40, n, dtype=np.int64)
    got = host(ex.sort_i64(dev(v, ex)))
    nbytes, _ = ex.sort_stats()
    assert (nbytes == 48 * n) == (kind == "narrow")
    assert np.array_equal(got, np.sort(v))
