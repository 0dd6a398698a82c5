"""GPU parity of nut_groupby_to_host: at large G the ordered path —
key-range partitions (GpRange), per-partition ordering, the result streamed to page-locked
host arrays chunk by chunk — must return exactly what nut_groupby + nut_groups_to_host
return (the hashed path + device ordering), and the oracle's groups: keys, counts, MIN /
MAX bit-exact, f64 sums within F64_SUM_RTOL (exact for dyadic values).  Shapes it does not
take (clustered keys, pageable outputs, the option off) fall back and give the same result;
heavy keys stay on it: keys the sample sees often (together >= 5 % of it) are aggregated in
the heavy-key pass before the partition levels (heavy.hpp), the excess of the others goes
through the overflow arenas."""
import numpy as np
import pytest
import torch

from helpers import F64_SUM_RTOL, rel_err
from test_gpu_exec import AGGS4, dev, gb_query

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max
N = (1 << 24) + 4099  # the ordered path starts at 2^24 rows


def pinned(rows, cols):
    return torch.empty((rows, cols), dtype=torch.int64, pin_memory=True).numpy()


def run_to_host(ex, q, hint, rows=None, pin=True):
    rows = rows or 2 * hint
    if pin:
        out = (pinned(rows, 1), pinned(rows, 4))
    else:
        out = (np.empty((rows, 1), np.int64), np.empty((rows, 4), np.int64))
    k, w = ex.groupby_to_host(q, group_hint=hint, out=out)
    path = ex.groupby_stats()["path"]
    if path != "partitioned_ordered":
        path += ":" + ex.groupby_declined()
    return k.copy(), w.copy(), path


def check(keys, words, ok, ow, sums_exact=False):
    assert np.array_equal(keys, ok)
    if sums_exact:
        assert np.array_equal(words[:, 0], ow[:, 0])
    else:
        assert rel_err(words[:, 0].view(np.float64), ow[:, 0].view(np.float64)) <= F64_SUM_RTOL
    assert np.array_equal(words[:, 1:], ow[:, 1:])


@pytest.mark.parametrize("G,dyadic", [(2_000_000, False), (3_000_000, True)])
def test_ordered_vs_oracle_and_hashed(ex, orc, G, dyadic):
    key = orc.gen_column(2, 0x61, N, a=G)
    val = orc.gen_column(3 if dyadic else 4, 0x62, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, G)
    assert path == "partitioned_ordered"
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    assert len(k) == len(ok) > 0.99 * G
    check(k, w, ok, ow, sums_exact=dyadic)
    # the hashed path + device ordering: the same groups, counts, MIN / MAX
    g = ex.groupby(q, group_hint=G)
    hk, hw = g.to_host_words()
    g.free()
    assert np.array_equal(hk, k)
    assert np.array_equal(hw[:, 1:], w[:, 1:])
    if dyadic:
        assert np.array_equal(hw, w)


def check_signed(keys, words, ok, ow, absum):
    """f64 sums of signed values: within F64_SUM_RTOL of the group's sum of |value| (the sums
    may cancel, so a relative bound on the sum itself does not apply); the rest exact."""
    assert np.array_equal(keys, ok)
    a, b = words[:, 0].view(np.float64), ow[:, 0].view(np.float64)
    assert np.all(np.abs(a - b) <= F64_SUM_RTOL * absum[:, 0].view(np.float64) + 1e-300)
    assert np.array_equal(words[:, 1:], ow[:, 1:])


def test_ordered_extreme_keys(ex, orc):
    """INT64_MIN (the tables' empty marker) and INT64_MAX each on 1/1000 of the rows, signed
    values and -0.0: the edge cells clamp, the order holds, and both heavy keys' excess
    rows go through the overflow arenas (the call stays on the ordered path)."""
    rng = np.random.default_rng(7)
    pool = rng.integers(I64_MIN, I64_MAX, 2_000_000, dtype=np.int64)
    pool[:4] = [I64_MIN, I64_MAX, I64_MIN + 1, I64_MAX - 1]
    key = pool[rng.integers(0, len(pool), N)]
    key[::1000] = I64_MIN
    key[1::1000] = I64_MAX
    val = rng.standard_normal(N)
    val[::97] = -0.0
    G = len(np.unique(key))
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, G)
    assert path == "partitioned_ordered"
    assert ex.groupby_overflow_rows() > 0 and ex.groupby_heavy() == (0, 0)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    _, absum = orc.groupby([key], [(0, 0, (0,))], values=[np.abs(val)])
    check_signed(k, w, ok, ow, absum)
    assert k[0, 0] == I64_MIN and k[-1, 0] == I64_MAX


def test_ordered_extreme_heavy_keys(ex, orc):
    """INT64_MIN and INT64_MAX on 4 % of the rows each, signed values: both go through the
    heavy-key pass (INT64_MIN is the hash tables' empty marker; the pass's set indexes its
    keys instead), the rest through the levels."""
    rng = np.random.default_rng(17)
    pool = rng.integers(I64_MIN, I64_MAX, 2_000_000, dtype=np.int64)
    key = pool[rng.integers(0, len(pool), N)]
    key[::25] = I64_MIN
    key[1::25] = I64_MAX
    val = rng.standard_normal(N)
    val[::97] = -0.0
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, len(np.unique(key)))
    assert path == "partitioned_ordered"
    hk, hr = ex.groupby_heavy()
    assert hk >= 2 and hr >= 2 * (N // 25)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    _, absum = orc.groupby([key], [(0, 0, (0,))], values=[np.abs(val)])
    check_signed(k, w, ok, ow, absum)
    assert k[0, 0] == I64_MIN and k[-1, 0] == I64_MAX


@pytest.mark.parametrize("share", [0.003, 0.02, 0.1])
def test_ordered_heavy_key(ex, orc, share):
    """One key on `share` of the rows: 0.3 % passes level 0 and overflows its level-1 region
    (the aggregation must not read past the region, and the result must hold);
    2 % overflows level 0 too — their excess is aggregated from the arenas and folded into
    the ordered result; 10 % (>= 5 % of the sample) goes through the heavy-key pass.  Same
    groups as the oracle, ordered path kept."""
    G = 2_000_000
    key = orc.gen_column(2, 0x6A, N, a=G)
    rng = np.random.default_rng(11)
    heavy = rng.random(N) < share
    key[heavy] = key[12345]
    val = orc.gen_column(3, 0x6B, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, G)
    assert path == "partitioned_ordered"
    if share >= 0.05:
        hk, hr = ex.groupby_heavy()  # (a key whose few rows the sample hit 4 times may join it)
        assert hk >= 1 and hr >= int((key == key[12345]).sum())
        assert ex.groupby_overflow_rows() == 0  # (exact layout behind the heavy pass)
    else:
        assert ex.groupby_overflow_rows() > 0 and ex.groupby_heavy() == (0, 0)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check(k, w, ok, ow, sums_exact=True)


@pytest.mark.parametrize("heavy_pass", [1, 2, 0])
def test_ordered_skew_generator(ex, orc, opts, heavy_pass):
    """Zipf-like keys (GEN_SKEW_KEY: pool index i on ~1/i of the rows, the top key ~6 %)
    on the ordered path vs the indexed oracle of the same generator: with the heavy-key pass
    (the default: the sample's frequent keys aggregated before the levels, whose regions are
    then laid out from exact per-cell counts — no overflow), with the pass but capped levels
    (gb_heavy = 2: the rest's excess through the overflow arenas), and without it (every
    excess through the arenas)."""
    from nutdb_amd import _lib as L
    opts(gb_heavy=heavy_pass)
    G = 4_000_000
    key = ex.gen_column(L.GEN_SKEW_KEY, 0x51, N, a=G)
    val = ex.gen_column(L.GEN_DYADIC, 0x52, N)
    q = gb_query(key, val)
    hint = int(orc.groupby_pool_dyadic(G, N, key_seed=0x51, val_seed=0x52, kind=7)[0].shape[0])
    k, w, path = run_to_host(ex, q, hint)
    ok, ow = orc.groupby_pool_dyadic(G, N, key_seed=0x51, val_seed=0x52, kind=7)
    assert path == "partitioned_ordered"
    hk, hr = ex.groupby_heavy()
    if heavy_pass:
        assert hk > 100 and hr > N // 4
        assert (ex.groupby_overflow_rows() == 0) == (heavy_pass == 1)
    else:
        assert (hk, hr) == (0, 0) and ex.groupby_overflow_rows() > 0
    assert np.array_equal(k, ok) and np.array_equal(w.view(np.uint64), ow)


@pytest.mark.parametrize("skew", [False, True])
def test_ordered_narrow_level1(ex, orc, opts, skew):
    """Level 1 at 512-thread scatter workgroups (NUT_OPT_GB_L1_THREADS = 512: 8 Ki-record
    tiles): the same groups, bit-exact, uniform pool keys and Zipf-like keys."""
    from nutdb_amd import _lib as L
    opts(gb_l1_threads=512)
    G = 4_000_000
    kind = L.GEN_SKEW_KEY if skew else L.GEN_POOL_KEY
    key = ex.gen_column(kind, 0x53, N, a=G)
    val = ex.gen_column(L.GEN_DYADIC, 0x54, N)
    ok, ow = orc.groupby_pool_dyadic(G, N, key_seed=0x53, val_seed=0x54, kind=kind)
    k, w, path = run_to_host(ex, gb_query(key, val), int(ok.shape[0]))
    assert path == "partitioned_ordered"
    assert np.array_equal(k, ok) and np.array_equal(w.view(np.uint64), ow)


def test_ordered_i64_values(ex, orc):
    from nutdb_amd import Agg, AggQuery
    rng = np.random.default_rng(8)
    G = 2_000_000
    key = orc.gen_column(2, 0x63, N, a=G)
    val = rng.integers(-(1 << 40), 1 << 40, N, dtype=np.int64)
    q = AggQuery(keys=[dev(key, ex)], values=[dev(val, ex)],
                 aggs=[Agg("sum", "col", (0,)), Agg("count"), Agg("min", "col", (0,)), Agg("max", "col", (0,))])
    k, w, path = run_to_host(ex, q, G)
    assert path == "partitioned_ordered"
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    assert np.array_equal(k, ok) and np.array_equal(w, ow)


def test_half_rows_on_one_key(ex, orc):
    """Half the rows on one key: the level-0 arena takes most of them (or, exhausted,
    the call falls back to the hashed path); either way the same result."""
    G = 2_000_000
    key = orc.gen_column(2, 0x64, N, a=G)
    key[::2] = key[1]
    val = orc.gen_column(3, 0x65, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, G)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check(k, w, ok, ow, sums_exact=True)


def test_clustered_keys_declined_up_front(ex, orc):
    """Half the distinct keys inside 1/2^20 of the sampled range would overfill one
    partition's table: the sample admission declines before any work (hashed path)."""
    G = 2_000_000
    rng = np.random.default_rng(13)
    pool = np.concatenate([rng.integers(I64_MIN, I64_MAX, G // 2, dtype=np.int64),
                           rng.integers(0, 1 << 43, G // 2, dtype=np.int64)])
    key = pool[rng.integers(0, G, N)]
    val = orc.gen_column(3, 0x6C, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, len(np.unique(key)))
    assert path == "partitioned_direct:clustered"
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check(k, w, ok, ow, sums_exact=True)


def test_pageable_and_option_off_fall_back(ex, orc, opts):
    G = 2_000_000
    key = orc.gen_column(2, 0x66, N, a=G)
    val = orc.gen_column(3, 0x67, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    k, w, path = run_to_host(ex, q, G, pin=False)
    assert path == "partitioned_direct:shape"
    check(k, w, ok, ow, sums_exact=True)
    opts(gb_ordered=0)
    k, w, path = run_to_host(ex, q, G)
    assert path == "partitioned_direct:shape"
    check(k, w, ok, ow, sums_exact=True)


def test_capacity_and_auto_size(ex, orc):
    from nutdb_amd._lib import NUT_ERR_CAPACITY, NutError
    G = 2_000_000
    key = orc.gen_column(2, 0x68, N, a=G)
    val = orc.gen_column(3, 0x69, N)
    q = gb_query(dev(key, ex), dev(val, ex))
    with pytest.raises(NutError) as ei:
        ex.groupby_to_host(q, group_hint=G, out=(pinned(G // 2, 1), pinned(G // 2, 4)))
    assert ei.value.status == NUT_ERR_CAPACITY
    k, w = ex.groupby_to_host(q, group_hint=G // 4)  # library-made arrays, resized once
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check(k, w, ok, ow, sums_exact=True)


def test_ordered_heavy_pass_two_value_columns(ex, orc):
    """The heavy-key pass with two value arrays (its NV = 2 kernel) and five aggregates —
    SUM / MIN / MAX of an i64 column, SUM / MAX of an f64 column, COUNT — over Zipf-like
    keys: heavy keys' i64 MIN / MAX and f64 MAX travel through its accumulators, the rest
    through the levels; every word bit-exact (dyadic f64 values)."""
    from nutdb_amd import Agg, AggQuery
    from nutdb_amd import _lib as L
    G = 6_000_000  # ~2.0e6 distinct keys: the ordered path needs >= 100 per range cell
    key = ex.gen_column(L.GEN_SKEW_KEY, 0x71, N, a=G)
    fv = ex.gen_column(L.GEN_DYADIC, 0x72, N)
    rng = np.random.default_rng(72)
    iv_h = rng.integers(-(1 << 40), 1 << 40, N, dtype=np.int64)
    iv = dev(iv_h, ex)
    q = AggQuery(keys=[key], values=[iv, fv],
                 aggs=[Agg("sum", "col", (0,)), Agg("min", "col", (0,)), Agg("max", "col", (0,)),
                       Agg("sum", "col", (1,)), Agg("max", "col", (1,)), Agg("count")])
    kh = key.cpu().numpy()
    hint = len(np.unique(kh))
    out = (pinned(2 * hint, 1), pinned(2 * hint, 6))
    k, w = ex.groupby_to_host(q, group_hint=hint, out=out)
    k, w = k.copy(), w.copy()
    assert ex.groupby_stats()["path"] == "partitioned_ordered", ex.groupby_declined()
    hk, hr = ex.groupby_heavy()
    assert hk > 50 and hr > N // 5
    ok, ow = orc.groupby([kh], [(0, 0, (0,)), (2, 0, (0,)), (3, 0, (0,)), (0, 0, (1,)), (3, 0, (1,)), (1, 0, ())],
                         values=[iv_h, fv.cpu().numpy()])
    assert np.array_equal(k, ok) and np.array_equal(w.view(np.uint64), ow)


@pytest.mark.parametrize("nkeys", [1, 400])
def test_ordered_all_rows_heavy(ex, orc, nkeys):
    """few distinct keys under a large group_hint — every key is heavy
    (<= 2048 / aggregates of them), the heavy pass takes every row and no row is left for
    the partition levels (the division by the partition count that followed is gone): the
    heavy groups are the result, as the oracle's."""
    rng = np.random.default_rng(23)
    n = 1 << 25
    pool = rng.integers(I64_MIN, I64_MAX, max(nkeys, 2), dtype=np.int64)
    pool[1] = pool[0] + (1 << 40)  # (the sampled key range must span >= 2^16)
    key = pool[rng.integers(0, nkeys, n)] if nkeys > 1 else np.full(n, pool[0])
    if nkeys == 1:
        key[::2] = pool[1]
    val = orc.gen_column(3, 0x6C, n)
    q = gb_query(dev(key, ex), dev(val, ex))
    k, w, path = run_to_host(ex, q, 1 << 21, rows=1 << 12)
    ok, ow = orc.groupby([key], AGGS4, values=[val])
    check(k, w, ok, ow, sums_exact=True)
    if path == "partitioned_ordered":
        hk, hr = ex.groupby_heavy()
        assert hr == n and hk == len(ok)
