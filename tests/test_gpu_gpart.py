"""GPU parity of the partitioned aggregation path (csrc/gpart.hpp): spill
-> hash partitions (one or two 8-bit levels) -> one workgroup per partition.  The context
options gb_partition=1 / gb_levels force the path and its levels at test sizes (and every
test checks nut_ctx_groupby_stats names that path); results must equal the
oracle exactly as the on-chip path's do (f64 sums within F64_SUM_RTOL, exact for dyadic)."""
import numpy as np
import pytest

from helpers import F64_SUM_RTOL, OPCODE, rel_err
from test_gpu_exec import AGGS4, check_vs_oracle, dev, gb_query

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max


@pytest.fixture(params=[1, 2], ids=["levels1", "levels2"])
def gp(request, opts):
    opts(gb_partition=1, gb_levels=request.param)
    return request.param


@pytest.mark.parametrize("G,hint", [(1, 1), (1000, 1000), (100_000, 100_000), (2_000_000, 2_000_000),
                                    (100_000, 0)])
def test_gp_cardinalities(ex, orc, gp, G, hint):
    n = 3_000_017
    key = orc.gen_column(2, 0x51, n, a=G)
    val = orc.gen_column(4, 0x52, n)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=hint)
    st = ex.groupby_stats()
    assert (st["path"], st["levels"]) == ("partitioned_direct", gp)
    if G >= 100_000:  # (very few keys per partition may overflow a 2x share: histogram layout)
        assert st["optimistic"]
    if G == 1:
        assert not st["optimistic"]
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    assert len(g) == len(ok)
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


def test_gp_dyadic_exact_and_predicate(ex, orc, gp):
    n = 2_000_003
    key = orc.gen_column(2, 0x51, n, a=300_000)
    val = orc.gen_column(3, 0x52, n)  # dyadic: every sum exact
    preds = [(dev(val, ex), "<", 6000.0)]
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex), preds), group_hint=300_000)
    assert ex.groupby_stats()["path"] == "partitioned_spill"
    ok, ow = orc.groupby([key], AGGS4, values=[val], preds=[(val, OPCODE["<"], 6000.0)])
    keys, words = g.to_host_words()
    assert np.array_equal(keys, ok) and np.array_equal(words, ow)


def test_gp_extreme_keys_and_negative_zero(ex, orc, gp):
    rng = np.random.default_rng(3)
    n = 400_000
    key = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64) // 1000 * 1000
    key[::7] = I64_MIN
    key[::11] = I64_MAX
    key[::13] = np.int64(-9223372036854775808 + 0)  # the table's empty marker
    val = rng.standard_normal(n)
    val[::100] = -0.0
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=len(np.unique(key)))
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


def test_gp_two_keys_preds_exprs(ex, orc, gp):
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(11)
    n = 1_000_001
    k1 = rng.integers(-3000, 4000, n).astype(np.int64)
    k2 = rng.integers(0, 70, n).astype(np.int64) * 1_000_000_007
    a = rng.random(n)
    b = rng.random(n)
    c = rng.random(n)
    f = rng.integers(0, 100, n).astype(np.int64)
    q = AggQuery(keys=[dev(k1, ex), dev(k2, ex)], values=[dev(a, ex), dev(b, ex), dev(c, ex)],
                 preds=[(dev(f, ex), ">=", 10), (dev(a, ex), "<", 0.9)],
                 aggs=[Agg("sum", "mul", (0, 1)), Agg("sum", "mul_1m_1p", (0, 1, 2)), Agg("min", "sub", (1, 2)),
                       Agg("count"), Agg("max", "add", (0, 2))])
    g = ex.groupby(q, group_hint=300_000)
    ok, ow = orc.groupby([k1, k2], [(0, 1, (0, 1)), (0, 5, (0, 1, 2)), (2, 3, (1, 2)), (1, 0, ()), (3, 2, (0, 2))],
                         values=[a, b, c], preds=[(f, OPCODE[">="], 10), (a, OPCODE["<"], 0.9)])
    check_vs_oracle(g, ok, ow, ["sum_f64", "sum_f64", "i", "i", "i"])


def test_gp_i64_wrap(ex, orc, gp):
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(5)
    n = 500_003
    key = rng.integers(0, 90_000, n).astype(np.int64)
    v = rng.integers(I64_MIN, I64_MAX, n, dtype=np.int64)
    q = AggQuery(keys=[dev(key, ex)], values=[dev(v, ex)],
                 aggs=[Agg("sum", "col", (0,)), Agg("min", "col", (0,)), Agg("max", "col", (0,)), Agg("count")])
    g = ex.groupby(q, group_hint=90_000)
    ok, ow = orc.groupby([key], [(0, 0, (0,)), (2, 0, (0,)), (3, 0, (0,)), (1, 0, ())], values=[v])
    check_vs_oracle(g, ok, ow, ["i", "i", "i", "i"])


@pytest.mark.parametrize("seed", range(4))
def test_gp_expression_programs_with_masks(ex, gp, seed):
    """Expression mode through the spill: masked COUNT is staged as 0/1, a masked-out value
    as its aggregate's identity — the groups and words equal the numpy oracle's."""
    from test_gpu_expr import Gen, make_table, run_both
    rng = np.random.default_rng(2000 + seed)
    n = 300_007
    cols, ic, fc = make_table(rng, n)
    g = Gen(rng, ic, fc)
    keys = [rng.integers(0, 50_000, n).astype(np.int64)]
    if seed % 2:
        keys.append(rng.integers(0, 3, n).astype(np.int64))
    where = g.bool_(2) if seed != 3 else None
    aggs = [("sum", g.int_(3), None), ("count", None, g.bool_(2)), ("max", g.f64_(2), g.bool_(1)),
            ("min", g.int_(2), g.bool_(1))]
    gk, gw, ok, ow, types = run_both(ex, keys, cols, where, aggs, 50_000)
    assert np.array_equal(gk, ok)
    assert np.array_equal(gw, ow), (seed, np.argwhere(gw != ow)[:5])


def test_gp_empty_and_all_rejected(ex, orc, gp):
    key = np.arange(5000, dtype=np.int64)
    val = np.ones(5000)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex), [(dev(key, ex), "<", -5)]), group_hint=5000)
    assert len(g) == 0


def test_gp_table_growth(ex, orc, opts):
    """A hint far below the real group count: the partitioned pass grows the table and
    re-runs only the per-partition aggregation."""
    opts(gb_partition=1)
    n = 2_000_000
    key = orc.gen_column(2, 0x51, n, a=500_000)
    val = orc.gen_column(4, 0x52, n)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=1000)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check_vs_oracle(g, ok, ow, ["sum_f64", "i", "i", "i"])


@pytest.mark.parametrize("levels", ["1", "2"])
@pytest.mark.parametrize("opt", ["0", "1"])
def test_gp_optimistic_layout_and_fallback(ex, orc, opts, opt, levels):
    """Direct partitioning whose first level has no histogram pass (gb_optimistic=1, the
    default): each of the 256 level-0 partitions owns twice its even share of rows.  Uniform keys fit; a heavy
    key (half the rows) overflows its partition, whose runs go to the scratch rows, and the
    level runs again with a histogram.  Both layouts equal the oracle bit for bit."""
    opts(gb_partition=1, gb_levels=int(levels), gb_optimistic=int(opt))
    n = 3_000_017
    for heavy in (False, True):
        key = orc.gen_column(2, 0x61, n, a=100_000)
        if heavy:
            key[::2] = 12345
        val = orc.gen_column(3, 0x62, n)  # dyadic: every sum exact
        g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=100_000)
        st = ex.groupby_stats()
        assert st["path"] == "partitioned_direct" and st["levels"] == int(levels)
        assert st["optimistic"] == (opt == "1" and not heavy)
        assert st["capped_levels"] == (1 if opt == "1" and not heavy else 0)  # (G = 1e5: level 1 histogram)
        ok, ow = orc.groupby([key], AGGS4, values=[val])
        keys, words = g.to_host_words()
        assert np.array_equal(keys, ok) and np.array_equal(words, ow), heavy


def _owner_hash(k):
    """common.hpp owner_hash(k, 0, 1) = mix64(k ^ 0x6A09E667F3BCC908), numpy uint64"""
    z = k.astype(np.uint64) ^ np.uint64(0x6A09E667F3BCC908)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


@pytest.mark.parametrize("bits1", [8, 6])
def test_gp_capped_level1_fallback(ex, orc, opts, bits1):
    """Two capped levels (offered from 6.5M expected groups: hint 1e7 over ~3M distinct
    keys): a key hash whose SECOND byte is skewed (30% of the rows on keys whose level-1
    digit is 7, spread over every level-0 digit) keeps level 0 capped and overflows level
    1, which runs again with a histogram; uniform keys keep both capped.  Both equal the
    oracle bit for bit."""
    opts(gb_partition=1, gb_levels=2, gb_optimistic=1, gb_l1_bits=bits1)
    n = 3_000_017
    rng = np.random.default_rng(17)
    cand = rng.integers(-2**62, 2**62, 4_000_000).astype(np.int64)
    sub7 = cand[((_owner_hash(cand) >> np.uint64(48)) & np.uint64(255)) == 7][:2000]
    assert len(sub7) == 2000 and len(np.unique(_owner_hash(sub7) >> np.uint64(56))) > 200
    for skew in (False, True):
        key = orc.gen_column(1, 0x63, n)  # distinct keys
        if skew:
            m = rng.random(n) < 0.3
            key[m] = rng.choice(sub7, int(m.sum()))
        val = orc.gen_column(3, 0x64, n)
        g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=10_000_000)
        st = ex.groupby_stats()
        assert (st["path"], st["levels"], st["optimistic"]) == ("partitioned_direct", 2, True)
        assert st["capped_levels"] == (1 if skew else 2), st
        ok, ow = orc.groupby([key], AGGS4, values=[val])
        keys, words = g.to_host_words()
        assert np.array_equal(keys, ok) and np.array_equal(words, ow), skew


def test_ordered_result_bucket_index(ex, orc):
    """Large one-key results are ordered on the device: sort of the unique keys, then each
    group binary-searches its bucket of a 2^20-bucket index over (k - min) >> shift.  Key
    sets with a small range (shift 0, consecutive ids), two clusters 2^62 apart (most
    buckets empty) and negative keys all come back in key order with their sums."""
    rng = np.random.default_rng(11)
    cases = {"consecutive": np.arange(-50_000, 150_000, dtype=np.int64),
             "two_clusters": np.concatenate([np.arange(100_000, dtype=np.int64) - 2**62,
                                             np.arange(100_000, dtype=np.int64) + 2**62]),
             "full_range": rng.integers(I64_MIN, I64_MAX, 300_000, dtype=np.int64)}
    for name, uniq in cases.items():
        key = np.repeat(uniq, 3)
        rng.shuffle(key)
        val = (np.abs(key) % 1000).astype(np.float64)
        g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=len(uniq))
        ok, ow = orc.groupby([key], AGGS4, values=[val])
        keys, words = g.to_host_words()
        assert np.array_equal(keys, ok) and np.array_equal(words, ow), name


def test_gp_dense_partitions_and_fallback(ex, orc, opts):
    """Two levels leave one workgroup per partition, whose groups are final: they are
    appended to the table unhashed (gb_dense, the default).  A partition with more groups
    than its workgroup's table admits (a hint far too small) reruns with the hashed merge;
    accumulating into a dense result rehashes it first.  All equal the oracle."""
    opts(gb_partition=1, gb_levels=2)
    n = 4_000_037
    key = orc.gen_column(1, 0x65, n)  # distinct keys
    key[::3] = key[1::3][: len(key[::3])]  # and some repeats
    val = orc.gen_column(3, 0x66, n)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    for hint in (n, 10):
        for dense in (1, 0):
            opts(gb_dense=dense)
            g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=hint)
            keys, words = g.to_host_words()
            assert np.array_equal(keys, ok) and np.array_equal(words, ow), (hint, dense)
    # accumulate more rows into a dense result
    opts(gb_dense=1)
    g = ex.groupby(gb_query(dev(key, ex), dev(val, ex)), group_hint=n)
    from nutdb_amd import Agg, AggQuery
    key2 = np.concatenate([orc.gen_column(2, 0x67, 500_000, a=1000), key[:1000]])
    val2 = orc.gen_column(3, 0x68, len(key2))
    ones = np.ones(len(key2), dtype=np.int64)  # COUNT partials merge as sums
    ex.accumulate(AggQuery(keys=[dev(key2, ex)], values=[dev(val2, ex), dev(ones, ex)],
                           aggs=[Agg("sum", "col", (0,)), Agg("sum", "col", (1,)), Agg("min", "col", (0,)),
                                 Agg("max", "col", (0,))]), g)
    ok2, ow2 = orc.groupby([np.concatenate([key, key2])], AGGS4, values=[np.concatenate([val, val2])])
    keys, words = g.to_host_words()
    assert np.array_equal(keys, ok2) and np.array_equal(words, ow2)
