"""GPU: Float64 single-column scans and ORDER BY through plan lowering (row B1), vs numpy.

`SELECT f FROM t [WHERE f <cmp> k] [ORDER BY f [DESC]] [LIMIT n]` over a Float64 column
(`Literal::Float`, /root/reference/src/parser/ast/item.rs:89-101; ORDER BY,
/root/reference/src/parser/ast/query.rs:86-90).  The reference executes nothing, so the
semantics are the build's:
  - WHERE compares in f64 (IEEE: -0.0 == +0.0, NaN fails every comparison but !=);
  - ORDER BY sorts by the IEEE total order: -NaN < -inf < ... < -0.0 < +0.0 < ... < +inf
    < +NaN (DESC: the reverse), i.e. by int64 words whose set sign bit flips the other 63.
Results are compared bit for bit (the order map is a bijection, so ties are bit-equal).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SPECIALS = np.array([0.0, -0.0, np.inf, -np.inf, 1.5, -1.5, 2.0, -2.0, 1.0, 5e-324, -5e-324,
                     np.finfo(np.float64).max, -np.finfo(np.float64).max], dtype=np.float64)


def order_key(f):
    b = f.view(np.int64)
    return b ^ ((b >> 63) & np.int64(0x7FFFFFFFFFFFFFFF))


def total_sort(f, desc=False):
    idx = np.argsort(order_key(f), kind="stable")
    return f[idx[::-1]] if desc else f[idx]


def column(n, seed, nan=False):
    rng = np.random.default_rng(seed)
    f = rng.integers(-4000, 4000, n) / 1000.0  # negatives, exact 1.5 / 2.0 hits
    f[rng.integers(0, n, n // 50)] = 0.0
    f[rng.integers(0, n, n // 50)] = -0.0
    f[rng.integers(0, n, n // 200)] = np.inf
    f[rng.integers(0, n, n // 200)] = -np.inf
    f[: len(SPECIALS)] = SPECIALS
    if nan:
        f[rng.integers(0, n, n // 300)] = np.nan
        f[rng.integers(0, n, n // 300)] = -np.nan  # sign-set quiet NaN
        f[7] = np.float64("nan")
    return f


def bits_equal(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def run(ex, sql, f):
    got = ex.sql(sql, {"f": torch.from_numpy(f).to(ex.device)})
    assert list(got) == ["f"]
    assert got["f"].dtype == np.float64
    return got["f"]


@pytest.mark.parametrize("n", [1, 13, 100_003, 1_000_003])
def test_select_f64_column(ex, n):
    f = column(max(n, len(SPECIALS)), 1)[:n] if n >= len(SPECIALS) else SPECIALS[:n].copy()
    assert bits_equal(run(ex, "select f from t", f), f)


@pytest.mark.parametrize("pred,fn", [
    ("f < 2", lambda f: f < 2),
    ("f < 1.5", lambda f: f < 1.5),
    ("f <= 1.5", lambda f: f <= 1.5),
    ("f > -1.5", lambda f: f > -1.5),
    ("f >= 0", lambda f: f >= 0),        # -0.0 passes: it equals 0
    ("f = 0", lambda f: f == 0),          # both zeros
    ("f != 2", lambda f: f != 2),         # NaN passes !=
    ("0.5 > f", lambda f: f < 0.5),       # mirrored
    ("f between -1 and 1", lambda f: (f >= -1) & (f <= 1)),
    ("f < 1" + "0" * 400 + ".5", lambda f: f < np.inf),  # the decimal rounds to +inf (no exponent literals)
])
@pytest.mark.parametrize("nan", [False, True])
def test_where_f64(ex, pred, fn, nan):
    f = column(300_007, 2, nan)
    with np.errstate(invalid="ignore"):
        want = f[fn(f)]
    assert bits_equal(run(ex, f"select f from t where {pred}", f), want)


@pytest.mark.parametrize("n", [0, 1, 5, 4099, 1_000_003, 3_000_017])
@pytest.mark.parametrize("desc", [False, True])
def test_order_by_f64(ex, n, desc):
    f = column(max(n, 64), 3, nan=True)[:n]
    got = run(ex, "select f from t order by f" + (" desc" if desc else ""), f)
    assert bits_equal(got, total_sort(f, desc))
    if n > 64:  # sanity: the numbers (NaNs aside) in order, the infinities at their ends
        num = got[~np.isnan(got)]
        fin = num[np.isfinite(num)]
        assert np.all(np.diff(fin) <= 0) if desc else np.all(np.diff(fin) >= 0)
        lo, hi = (num[-1], num[0]) if desc else (num[0], num[-1])
        assert lo == -np.inf and hi == np.inf


@pytest.mark.parametrize("limit", [1, 100, 5000])
@pytest.mark.parametrize("desc", [False, True])
def test_order_by_f64_limit(ex, limit, desc):
    f = column(2_000_003, 4, nan=False)
    got = run(ex, f"select f from t order by f{' desc' if desc else ''} limit {limit}", f)
    assert bits_equal(got, total_sort(f, desc)[:limit])


def test_order_by_f64_with_where_and_offset(ex):
    f = column(1_000_003, 5, nan=True)
    got = run(ex, "select f from t where f < 2 order by f desc limit 100 offset 7", f)
    with np.errstate(invalid="ignore"):
        sel = f[f < 2]
    assert bits_equal(got, total_sort(sel, True)[7:107])


def test_order_by_f64_all_equal_and_zeros(ex):
    z = np.where(np.arange(200_000) % 3 == 0, -0.0, 0.0)
    assert bits_equal(run(ex, "select f from t order by f", z), total_sort(z))
    assert bits_equal(run(ex, "select f from t order by f desc", z), total_sort(z, True))
    c = np.full(70_001, -3.25)
    assert bits_equal(run(ex, "select f from t order by f", c), c)


def test_f64_scan_with_int_column_where(ex):
    """a float64 projection under an int64 WHERE and an int64 projection ordered by a
    float64 column (the row-id scan)"""
    rng = np.random.default_rng(6)
    n = 500_009
    f = column(n, 6)
    a = rng.integers(-100, 100, n)
    cols = {"f": torch.from_numpy(f).to(ex.device), "a": torch.from_numpy(a).to(ex.device)}
    got = ex.sql("select f from t where a < 10", cols)
    assert bits_equal(got["f"], f[a < 10])
    got = ex.sql("select a from t order by f desc, a", cols)
    idx = np.lexsort((a, -order_key(f)))  # DESC f: the reversed total order, then a
    assert np.array_equal(got["a"], a[idx])


def canon_words(f):
    """the executor's GROUP BY key words: -0.0 -> +0.0, every NaN -> +qNaN, then order_key"""
    g = np.where(f == 0, 0.0, f)
    g = np.where(np.isnan(g), np.float64("nan"), g)
    g = g.copy()
    g[np.isnan(g)] = np.frombuffer(np.uint64(0x7FF8000000000000).tobytes(), dtype=np.float64)[0]
    return order_key(g), g


@pytest.mark.parametrize("n", [1, 1000, 2_000_003])
def test_group_by_f64_key(ex, n):
    """GROUP BY a Float64 column: one group for -0.0 / +0.0 (reported +0.0), one for all
    NaNs (the quiet +NaN, last), groups in the IEEE total order; sums / counts exact"""
    rng = np.random.default_rng(8)
    f = column(max(n, 64), 8, nan=True)[:n]
    v = rng.integers(-1000, 1000, n)
    got = ex.sql("select f, count(*) as c, sum(v) as s, min(v) as lo from t group by f",
                 {"f": torch.from_numpy(f).to(ex.device), "v": torch.from_numpy(v).to(ex.device)})
    w, g = canon_words(f)
    uw, inv = np.unique(w, return_inverse=True)
    first = np.zeros(len(uw), dtype=np.int64)
    first[inv[::-1]] = np.arange(n)[::-1]
    assert bits_equal(got["f"], g[first])
    assert np.array_equal(got["c"], np.bincount(inv, minlength=len(uw)))
    assert np.array_equal(got["s"], np.bincount(inv, weights=v, minlength=len(uw)).astype(np.int64))
    lo = np.full(len(uw), np.iinfo(np.int64).max)
    np.minimum.at(lo, inv, v)
    assert np.array_equal(got["lo"], lo)


def test_group_by_f64_key_order_desc_having_and_distinct(ex):
    rng = np.random.default_rng(9)
    n = 500_009
    f = np.round(column(n, 9, nan=True), 1)
    v = rng.integers(0, 10, n)
    cols = {"f": torch.from_numpy(f).to(ex.device), "v": torch.from_numpy(v).to(ex.device)}
    w, g = canon_words(f)
    uw, inv = np.unique(w, return_inverse=True)
    cnt = np.bincount(inv, minlength=len(uw))
    first = np.zeros(len(uw), dtype=np.int64)
    first[inv[::-1]] = np.arange(n)[::-1]
    keys = g[first]
    got = ex.sql("select f, count(*) as c from t group by f having count(*) > 100 order by f desc limit 50", cols)
    keep = np.nonzero(cnt > 100)[0][::-1][:50]
    assert bits_equal(got["f"], keys[keep]) and np.array_equal(got["c"], cnt[keep])
    got = ex.sql("select distinct f from t", cols)
    assert bits_equal(got["f"], keys)


@pytest.mark.parametrize("signed", [False, True])
def test_group_by_f64_and_int_keys_packed(ex, signed):
    """packed key words (a computed key): an int64 column, a Float64 column and a%2.  The
    words of positive doubles span < 2^53 values, so all three share one word; doubles of
    both signs span ~2^63 words, so (f, z) take both words and a third key is refused"""
    rng = np.random.default_rng(10)
    n = 300_007
    a = rng.integers(0, 5, n)
    f = rng.integers(-3, 3, n) / 2.0 if signed else rng.integers(1, 8, n) / 2.0
    if signed:
        f[::17] = -0.0
    cols = {"a": torch.from_numpy(a).to(ex.device), "f": torch.from_numpy(f).to(ex.device)}
    w, g = canon_words(f)
    if signed:
        from nutdb_amd import NutError
        with pytest.raises(NutError, match="more than 2 x 63 bits"):
            ex.sql("select a, f, a % 2 as z, count(*) as c from t group by a, f, z", cols)
        got = ex.sql("select f, a % 2 as z, count(*) as c, sum(f) as s from t group by f, z", cols)
        tup = np.stack([w, a % 2], axis=1)
    else:
        got = ex.sql("select a, f, a % 2 as z, count(*) as c, sum(f) as s from t group by a, f, z", cols)
        tup = np.stack([a, w, a % 2], axis=1)
    u, inv = np.unique(tup, axis=0, return_inverse=True)
    inv = inv.ravel()
    if not signed:
        assert np.array_equal(got["a"], u[:, 0])
    assert np.array_equal(got["z"], u[:, -1])
    first = np.zeros(len(u), dtype=np.int64)
    first[inv[::-1]] = np.arange(n)[::-1]
    assert bits_equal(got["f"], g[first])
    assert np.array_equal(got["c"], np.bincount(inv, minlength=len(u)))
    assert np.array_equal(got["s"], np.bincount(inv, weights=f, minlength=len(u)))
