"""Pin the C oracle (oracle/liboracle.so) to the committed golden fixtures.

The fixtures come from numpy / pyarrow / math.fsum (tests/golden/make_golden.py),
independent of the oracle's C code.  CPU only.
"""
import numpy as np
import pytest

from helpers import F64_SUM_RTOL, OPCODE, fromhex, gen, multiset_hash, pos_hash, rel_err, wsum


def test_generator_matches_numpy(golden, orc):
    for case in golden["generator"]:
        v = orc.gen_column(case["kind"], case["seed"], case["n"], row0=case["row0"], a=case["a"],
                           b=case["b"], c=case["c"])
        assert [int(x) for x in v[:8].view(np.uint64)] == case["head"], case
        assert wsum(v) == case["wsum"], case


def test_generator_numpy_restatement(golden):
    # the numpy generator itself reproduces the fixture (guards the fixture script)
    for case in golden["generator"]:
        v = gen(case["kind"], case["seed"], case["n"], case["a"], case["b"], case["c"], case["row0"])
        assert wsum(v) == case["wsum"]


def test_filter(golden, orc):
    n = golden["filter"][0]["n"]
    col = orc.gen_column(0, 0x2A, n)
    for case in golden["filter"]:
        out = orc.filter_i64(col, OPCODE[case["op"]], case["k"])
        assert len(out) == case["count"], case["op"]
        assert [int(x) for x in out[:8]] == case["head"]
        assert [int(x) for x in out[-8:]] == case["tail"]
        assert pos_hash(out) == case["pos_hash"]


def test_filter_edges(orc):
    assert len(orc.filter_i64(np.array([], dtype=np.int64), 0, 5)) == 0
    v = np.array([5, -3, 7, 5, np.iinfo(np.int64).min, np.iinfo(np.int64).max], dtype=np.int64)
    for op, f in [(0, v < 5), (1, v <= 5), (2, v > 5), (3, v >= 5), (4, v == 5), (5, v != 5)]:
        assert np.array_equal(orc.filter_i64(v, op, 5), v[f])


@pytest.mark.parametrize("idx", range(5))
def test_groupby(golden, orc, idx):
    case = golden["groupby"][idx]
    n, G = case["n"], case["G"]
    key = orc.gen_column(2, 0x51, n, a=G)
    val = orc.gen_column(3 if case["dyadic"] else 4, 0x52, n)
    preds = [(val, OPCODE["<"], case["pred_val_lt"])] if case["pred_val_lt"] is not None else []
    keys, words = orc.groupby([key], [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,))], values=[val],
                              preds=preds)
    assert [int(k) for k in keys[:, 0]] == case["keys"]
    s = words[:, 0].view(np.float64)
    fs = fromhex(case["sum_fsum"])
    if case["dyadic"]:
        assert np.array_equal(s, fs)  # exact sums
    assert rel_err(s, fs) <= F64_SUM_RTOL
    assert [int(x) for x in words[:, 1]] == case["count"]
    assert np.array_equal(words[:, 2].view(np.float64), fromhex(case["min"]))
    assert np.array_equal(words[:, 3].view(np.float64), fromhex(case["max"]))


@pytest.mark.parametrize("idx", range(2))
def test_q1(golden, orc, idx):
    from nutdb_amd.workloads import Q1_COLS, Q1_DATE_K
    case = golden["q1"][idx]
    cols = [orc.gen(spec, case["n"], row0=case["row0"]) for spec in Q1_COLS]
    sd, rf, ls, qty, price, disc = cols
    keys, words = orc.groupby([rf, ls], [(0, 0, (0,)), (0, 0, (1,)), (0, 4, (1, 2)), (1, 0, ())],
                              values=[qty, price, disc], preds=[(sd, OPCODE["<="], Q1_DATE_K)])
    assert len(keys) == len(case["groups"])
    for (k, w, g) in zip(keys, words, case["groups"]):
        assert (int(k[0]), int(k[1])) == (g["returnflag"], g["linestatus"])
        assert int(w[3]) == g["count"]
        for j, name in enumerate(["sum_qty", "sum_price", "sum_disc_price"]):
            assert rel_err([w[j:j + 1].view(np.float64)[0]], [float.fromhex(g[name])]) <= F64_SUM_RTOL


def test_sort(golden, orc):
    case = golden["sort"][0]
    keys = orc.gen_column(1, 0x50, case["n"])
    out = orc.sort_i64(keys)
    assert [int(x) for x in out[:8]] == case["head"]
    assert [int(x) for x in out[-8:]] == case["tail"]
    assert pos_hash(out) == case["pos_hash"]
    assert orc.multiset_hash(keys) != 0 and multiset_hash(keys) == case["multiset_hash"]
    assert orc.multiset_hash(out) == orc.multiset_hash(keys)


def test_groupby_i64_sum_wraps_and_minmax(orc):
    big = np.iinfo(np.int64).max
    key = np.array([1, 1, 2, 2, 2], dtype=np.int64)
    v = np.array([big, 5, -4, 9, np.iinfo(np.int64).min], dtype=np.int64)
    keys, w = orc.groupby([key], [(0, 0, (0,)), (2, 0, (0,)), (3, 0, (0,)), (1, 0, ())], values=[v])
    assert list(keys[:, 0]) == [1, 2]
    sums = w[:, 0].view(np.int64)
    with np.errstate(over="ignore"):
        assert sums[0] == (np.int64(big) + np.int64(5))
    assert list(w[:, 1].view(np.int64)) == [5, np.iinfo(np.int64).min]
    assert list(w[:, 2].view(np.int64)) == [big, 9]
    assert list(w[:, 3].view(np.int64)) == [2, 3]


@pytest.mark.parametrize("groups,n,row0", [(1, 1000, 0), (1000, 200_000, 0), (100_000, 2_000_000, 12345),
                                           (3_000_000, 1_000_000, 7)])
def test_groupby_pool_indexed_matches_hash_oracle(orc, groups, n, row0):
    """The indexed dense-array oracle (the full-size config-3 checker, 1e9 rows x G up to
    1e7) equals the hash-table oracle on the same generated columns — including G > n,
    where some pool keys take no row and must be absent."""
    from nutdb_amd.workloads import groupby_cols
    ks, vs = groupby_cols(groups, dyadic=True)
    key, val = orc.gen(ks, n, row0=row0), orc.gen(vs, n, row0=row0)
    hk, hw = orc.groupby([key], [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,))], values=[val],
                         cap=min(groups, n))
    ik, iw = orc.groupby_pool_dyadic(groups, n, row0=row0, key_seed=ks[2], val_seed=vs[2])
    assert np.array_equal(ik, hk)
    assert np.array_equal(iw, hw)
    assert int(iw[:, 1].sum()) == n


@pytest.mark.parametrize("groups,nk,masked,skew", [(500_000, 1, False, False), (1_000_000, 1, True, False),
                                                   (300_000, 2, True, False), (20_000, 1, False, False),
                                                   (1_000_000, 1, False, True), (1_000_000, 2, True, True)])
def test_groupby_partitioned_merge_is_bitwise_the_table_merge(orc, groups, nk, masked, skew):
    """orc_groupby's key-range partitioned merge (large G: the CPU baseline's path) gives
    the per-thread-table merge's result bit for bit — keys, counts, i64 / f64 MIN / MAX and
    Neumaier f64 sums of non-dyadic values (the same per-group fold and merge order) —
    with a WHERE, a row mask and two keys; Zipf-like keys (skew) through the heavy-tuple
    split (keys holding >= 1/threads of the sample folded per thread chunk)."""
    n = (1 << 22) + 12345
    from nutdb_amd.workloads import groupby_cols
    ks, _ = groupby_cols(groups, dyadic=True, skew=skew)
    key = orc.gen(ks, n)
    keys = [key] if nk == 1 else [key, orc.gen_column(5, 0x3A, n, a=-3, b=7)]
    v = orc.gen_column(4, 0x55, n)              # unit f64: sums round
    iv = orc.gen_column(0, 0x56, n) - (1 << 61)  # signed i64
    aggs = [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,)), (0, 0, (1,)), (2, 0, (1,))]
    kw = {}
    if masked:
        kw = {"preds": [(iv, 0, 1 << 60)], "row_mask": (key & 7) != 3}
    a = orc.groupby(keys, aggs, values=[v, iv], **kw)
    b = orc.groupby(keys, aggs, values=[v, iv], method="tables", **kw)
    assert len(a[0]) > 1000
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("nthreads,share", [(16, 0.08), (8, 0.3), (4, 0.6)])
def test_groupby_heavy_tuples_split_is_bitwise(orc, nthreads, share):
    """Keys holding >= 1/threads of the rows: the range-partitioned
    merge folds them per thread chunk and merges the chunks' groups in order — still the
    per-thread-table merge's words bit for bit (non-dyadic f64 sums, i64 MIN / MAX, a WHERE)."""
    n = (1 << 22) + 777
    rng = np.random.default_rng(41)
    key = orc.gen_column(2, 0x71, n, a=1_000_000)
    hot = rng.random(n)
    key[hot < share] = key[3]
    key[(hot >= share) & (hot < 1.5 * share)] = key[99]  # a second, lighter heavy tuple
    v = orc.gen_column(4, 0x72, n)
    iv = orc.gen_column(0, 0x73, n) - (1 << 61)
    aggs = [(0, 0, (0,)), (1, 0, ()), (2, 0, (1,)), (3, 0, (0,))]
    kw = {"preds": [(iv, 0, 1 << 61)]}
    a = orc.groupby([key], aggs, values=[v, iv], nthreads=nthreads, **kw)
    b = orc.groupby([key], aggs, values=[v, iv], nthreads=nthreads, method="tables", **kw)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("groups", [6, 1000, 4096, 50_000])
def test_groupby_few_groups_gate_is_bitwise(orc, groups):
    """The few-groups gate ahead of the k-minimum-values sketch (every sampled key seen at
    least twice: the per-thread tables without hashing every row) and the sketch's path
    just above it give the per-thread-table merge's words bit for bit."""
    n = (1 << 22) + 5
    key = orc.gen_column(2, 0x81, n, a=groups)
    v = orc.gen_column(4, 0x82, n)
    aggs = [(0, 0, (0,)), (1, 0, ())]
    a = orc.groupby([key], aggs, values=[v], nthreads=4)
    b = orc.groupby([key], aggs, values=[v], nthreads=4, method="tables")
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert len(a[0]) <= groups
