"""GPU: computed projections of scans (SELECT a * 2 + b, toYYYYMMDD(d), CASE ... FROM t;
nut_eval_rows / select_kernel.hpp eval_kernel) and SQL NULLs in scan output — a
LEFT / RIGHT / FULL OUTER joined table's columns, a CASE branch without ELSE — returned as
masked arrays through nut_result_validity.  The shape of the reference fixture
tests/sql/10.sql (a LEFT JOIN chain projecting jh.job_id, toYYYYMMDD(e.hire_date), a CASE
over jh columns).  Expected values: numpy with the nut_prog semantics (oracle/expr.py for
date parts) and pandas merges for the joins."""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle.expr import date_part
from test_gpu_exec import dev

pytestmark = pytest.mark.gpu

NULL = np.iinfo(np.int64).min  # sentinel for comparing multisets of rows with NULLs


def on_dev(ex, t):
    return {k: dev(v, ex) for k, v in t.items()}


def filled(a, fill=NULL):
    """masked array (or plain) -> plain array with NULLs replaced by `fill`"""
    return np.ma.filled(a, fill) if np.ma.isMaskedArray(a) else np.asarray(a)


def rows_of(cols):
    """multiset of rows: lexicographically sorted list of tuples"""
    return sorted(zip(*[c.tolist() for c in cols]))


@pytest.fixture(scope="module")
def table():
    rng = np.random.default_rng(77)
    n = 300_001
    return {"a": rng.integers(-10**6, 10**6, n).astype(np.int64), "b": rng.random(n),
            "d": rng.integers(-800_000, 2_900_000, n).astype(np.int64), "k": rng.integers(0, 50, n).astype(np.int64)}


def test_computed_projections_vs_numpy(ex, table):
    t = table
    a, b, d = t["a"], t["b"], t["d"]
    got = ex.sql("select a * 2 + b as s, toYYYYMMDD(d) as ymd, toYYYYMM(d) as ym, a % 7 as m, a, "
                 "case when b > 0.5 then b end as cb, intDiv(a, 3) - k as q from t where a > 1000 and k < 40",
                 on_dev(ex, t))
    sel = (a > 1000) & (t["k"] < 40)
    assert got["a"].tolist() == a[sel].tolist()  # table order
    assert np.array_equal(got["s"], (a[sel] * 2).astype(np.float64) + b[sel])  # bit-exact f64
    assert got["ymd"].tolist() == date_part(d[sel], 7).tolist()
    assert got["ym"].tolist() == date_part(d[sel], 6).tolist()
    assert got["m"].tolist() == np.fmod(a[sel], 7).tolist()  # % truncates toward zero
    assert got["q"].tolist() == (np.trunc(a[sel] / 3).astype(np.int64) - t["k"][sel]).tolist()
    cb = got["cb"]
    assert np.ma.isMaskedArray(cb) and np.array_equal(cb.mask, ~(b[sel] > 0.5))
    assert np.array_equal(cb.compressed(), b[sel][b[sel] > 0.5])
    assert not np.ma.isMaskedArray(got["s"])  # no NULLs: a plain array


def test_computed_projections_order_limit_and_many(ex, table):
    t = table
    a = t["a"]
    # ORDER BY a plain column, LIMIT: the computed columns follow the sorted rows
    got = ex.sql("select a - 5 as x, k * k as kk from t where k = 3 order by a desc limit 100", on_dev(ex, t))
    sel = np.flatnonzero(t["k"] == 3)
    o = sel[np.argsort(-a[sel], kind="stable")][:100]
    assert got["x"].tolist() == (a[o] - 5).tolist() and got["kk"].tolist() == [9] * 100
    # LIMIT / OFFSET without ORDER BY: the first selected rows in table order
    got = ex.sql("select a + 1 as x from t where a < 0 limit 7 offset 3", on_dev(ex, t))
    assert got["x"].tolist() == (a[a < 0][3:10] + 1).tolist()
    # more than 8 computed projections: several evaluation launches
    items = ", ".join(f"a + {i} as c{i}" for i in range(11))
    got = ex.sql(f"select {items}, k from t where k = 7", on_dev(ex, t))
    for i in range(11):
        assert got[f"c{i}"].tolist() == (a[t["k"] == 7] + i).tolist()
    # nothing selected: empty (masked) columns
    got = ex.sql("select a * 2 as x, case when a > 0 then a end as y from t where a > 10000000", on_dev(ex, t))
    assert len(got["x"]) == 0 and len(got["y"]) == 0


def test_computed_projection_errors(ex, table):
    from nutdb_amd import NutError
    with pytest.raises(NutError, match="division by zero"):
        ex.sql("select intDiv(a, k - k) from t where a > 0", on_dev(ex, table))


def orders_lines(seed=5, no=4000, nl=12000):
    rng = np.random.default_rng(seed)
    orders = {"o_okey": rng.permutation(no).astype(np.int64) * 2, "o_cust": rng.integers(0, 700, no).astype(np.int64),
              "o_date": rng.integers(8000, 11000, no).astype(np.int64)}
    lines = {"l_okey": rng.integers(-200, 2 * no + 400, nl).astype(np.int64),
             "l_qty": rng.integers(1, 50, nl).astype(np.int64)}
    return orders, lines


def test_left_join_projects_nulls(ex):
    orders, lines = orders_lines()
    do, dl = pd.DataFrame(orders), pd.DataFrame(lines)
    got = ex.sql("select o_okey, l_qty, l_qty * 2 + o_cust as v, toYYYYMMDD(o_date) as day from orders "
                 "left join lineitem on o_okey = l_okey where o_cust < 500", on_dev(ex, orders),
                 right=on_dev(ex, lines))
    m = do[do.o_cust < 500].merge(dl, left_on="o_okey", right_on="l_okey", how="left")
    q = m.l_qty.to_numpy(dtype=float)
    want_v = np.where(np.isnan(q), NULL, np.nan_to_num(q).astype(np.int64) * 2 + m.o_cust.to_numpy())
    want = rows_of([m.o_okey.to_numpy(), np.where(np.isnan(q), NULL, np.nan_to_num(q).astype(np.int64)), want_v,
                    date_part(m.o_date.to_numpy(), 7)])
    assert np.ma.isMaskedArray(got["l_qty"]) and np.ma.isMaskedArray(got["v"])
    assert not np.ma.isMaskedArray(got["o_okey"]) and not np.ma.isMaskedArray(got["day"])
    assert int(got["l_qty"].mask.sum()) == int(np.isnan(q).sum()) > 0
    assert rows_of([filled(got[c]) for c in ("o_okey", "l_qty", "v", "day")]) == want


def test_right_and_full_join_project_nulls(ex):
    orders, lines = orders_lines(9, 3000, 8000)
    do, dl = pd.DataFrame(orders), pd.DataFrame(lines)
    for how, kw in (("right", "right join"), ("outer", "full outer join")):
        got = ex.sql(f"select o_okey, o_cust, l_okey, l_qty from orders {kw} lineitem on o_okey = l_okey",
                     on_dev(ex, orders), right=on_dev(ex, lines))
        m = do.merge(dl, left_on="o_okey", right_on="l_okey", how=how)
        want = rows_of([np.where(m[c].isna(), NULL, m[c].fillna(0)).astype(np.int64)
                        for c in ("o_okey", "o_cust", "l_okey", "l_qty")])
        assert rows_of([filled(got[c]) for c in ("o_okey", "o_cust", "l_okey", "l_qty")]) == want, how
        assert int(np.ma.getmaskarray(got["l_qty"]).sum()) == int(m.l_qty.isna().sum())
        assert int(np.ma.getmaskarray(got["o_okey"]).sum()) == int(m.o_okey.isna().sum())


def test_left_join_chain_projects_nulls(ex):
    """fixture 10's shape: INNER then LEFT steps, projecting columns (and expressions) of
    LEFT-joined tables, one of them reached through a NULL-extended ON key"""
    rng = np.random.default_rng(31)
    ne, nj, nh = 3000, 40, 5000
    emp = {"e_id": rng.permutation(ne).astype(np.int64), "e_job": rng.integers(0, nj, ne).astype(np.int64),
           "e_mgr": rng.integers(-1, ne, ne).astype(np.int64), "e_hire": rng.integers(9000, 12000, ne).astype(np.int64)}
    jobs = {"j_id": np.arange(nj, dtype=np.int64), "j_min": rng.integers(1000, 5000, nj).astype(np.int64)}
    hist = {"h_emp": rng.integers(0, 2 * ne, nh).astype(np.int64), "h_job": rng.integers(0, 2 * nj, nh).astype(np.int64),
            "h_level": rng.integers(0, 64, nh).astype(np.int64), "h_off": rng.integers(0, 4, nh).astype(np.int64)}
    jobs2 = {"jj_id": np.arange(nj, dtype=np.int64), "jj_max": rng.integers(5000, 9000, nj).astype(np.int64)}
    got = ex.sql("""select e_id, toYYYYMMDD(e_hire) as hired, j_min, h_job,
                           case h_level >> h_off when 1 then 10 when 2 then 20 else h_level * (h_off + 1 * 3 % 4) end
                             as level,
                           jj_max
                    from emp join jobs on e_job = j_id
                    left join hist on e_id = h_emp
                    left join jobs2 on h_job = jj_id
                    order by e_id""", on_dev(ex, emp),
                 right=[on_dev(ex, jobs), on_dev(ex, hist), on_dev(ex, jobs2)])
    m = (pd.DataFrame(emp).merge(pd.DataFrame(jobs), left_on="e_job", right_on="j_id")
         .merge(pd.DataFrame(hist), left_on="e_id", right_on="h_emp", how="left")
         .merge(pd.DataFrame(jobs2), left_on="h_job", right_on="jj_id", how="left"))
    assert got["e_id"].tolist() == sorted(m.e_id.tolist())  # ORDER BY a preserved column
    lv, off = m.h_level.to_numpy(dtype=float), m.h_off.to_numpy(dtype=float)
    lvi, offi = np.nan_to_num(lv).astype(np.int64), np.nan_to_num(off).astype(np.int64)
    sh = lvi >> offi
    level = np.where(sh == 1, 10, np.where(sh == 2, 20, lvi * (offi + 3)))
    want = rows_of([m.e_id.to_numpy(), date_part(m.e_hire.to_numpy(), 7), m.j_min.to_numpy(),
                    np.where(m.h_job.isna(), NULL, m.h_job.fillna(0)).astype(np.int64),
                    np.where(np.isnan(lv), NULL, level),
                    np.where(m.jj_max.isna(), NULL, m.jj_max.fillna(0)).astype(np.int64)])
    assert rows_of([filled(got[c]) for c in ("e_id", "hired", "j_min", "h_job", "level", "jj_max")]) == want
    assert int(np.ma.getmaskarray(got["jj_max"]).sum()) == int(m.jj_max.isna().sum()) > int(m.h_job.isna().sum())


def test_null_projection_rejections(ex):
    from nutdb_amd import NutError
    orders, lines = orders_lines(3, 500, 1500)
    o, l_ = on_dev(ex, orders), on_dev(ex, lines)
    with pytest.raises(NutError, match="IS \\[NOT\\] NULL"):
        ex.sql("select o_okey, case when l_qty is null then 0 else l_qty end from orders left join lineitem "
               "on o_okey = l_okey", o, right=l_)
    with pytest.raises(NutError, match="may only appear inside aggregates and projections"):
        ex.sql("select o_okey from orders left join lineitem on o_okey = l_okey where l_qty > 3", o, right=l_)


def test_select_star(ex, table):
    """SELECT * projects every bound column in binding order: the reference's criterion
    statement (tests/golden/sql/bench_short.sql) over a table, WHERE / ORDER BY / LIMIT."""
    from pathlib import Path
    sql = (Path(__file__).parent / "golden" / "sql" / "bench_short.sql").read_text()
    got = ex.sql(sql, on_dev(ex, table))
    assert list(got) == list(table)
    for c in table:
        assert np.array_equal(got[c], table[c]), c
    got = ex.sql("select * from t where k = 5 order by a desc limit 20", on_dev(ex, table))
    sel = np.flatnonzero(table["k"] == 5)
    o = sel[np.argsort(-table["a"][sel], kind="stable")][:20]
    for c in table:
        assert np.array_equal(got[c], table[c][o]), c


def test_select_star_typed_table(ex):
    from nutdb_amd.table import Table
    rng = np.random.default_rng(8)
    n = 10_007
    s = np.array(["lo", "mid", "hi"], dtype=object)[rng.integers(0, 3, n)]
    v = rng.integers(-50, 50, n)
    t = Table(ex, "CREATE TABLE t (s String, v Int32, f Float64)")
    f = rng.random(n)
    t.append(s=s, v=v.astype(np.int32), f=f)
    got = t.sql("select * from t where v > 10")
    m = v > 10
    assert list(got) == ["s", "v", "f"]
    assert got["s"].tolist() == s[m].tolist() and got["v"].tolist() == v[m].tolist()
    assert np.array_equal(got["f"], f[m])


FIXTURE10_NUMERIC = """SELECT
    e.employee_id AS `Employee #`,
    toYYYYMMDD(e.hire_date) AS `Hire Date`,
    e.commission_pct AS `Comission %`,
    jh.job_id AS `History Job ID`,
    case jh.level >> jh.offset
        when 0x1 then 1
        when 0x2 then 2
        when 0x3 then 3
        else jh.n * (jh.k + 1 * 3 % 4)
    end AS level,
    r.region_id AS region,
    dd.location_id AS hist_location
FROM employees AS e
JOIN jobs AS j
  ON e.job_id = j.job_id
LEFT JOIN employees AS m
  ON e.manager_id = m.employee_id
LEFT JOIN departments AS d
  ON d.department_id = e.department_id
LEFT JOIN employees AS dm
  ON d.manager_id = dm.employee_id
LEFT JOIN locations AS l
  ON d.location_id = l.location_id
LEFT JOIN countries AS c
  ON l.country_id = c.country_id
LEFT JOIN regions AS r
  ON c.region_id = r.region_id
LEFT JOIN job_history AS jh
  ON e.employee_id = jh.employee_id
LEFT JOIN jobs AS jj
  ON jj.job_id = jh.job_id
LEFT JOIN departments AS dd
  ON dd.department_id = jh.department_id
ORDER BY
  e.employee_id"""


def test_fixture10_join_chain(ex):
    """The reference fixture tests/sql/10.sql's FROM / JOIN chain verbatim (11 tables, three
    of them twice under other aliases, 9 LEFT steps, ON keys read from NULL-extended tables),
    its toYYYYMMDD and its CASE over jh columns, with the string items (`first_name + ' ' +
    last_name`, the 'A'..'F' branches) replaced by numeric ones.  Reference: pandas merges."""
    rng = np.random.default_rng(10)
    ne, nj, nd, nl, nc, nr, nh = 2000, 30, 60, 40, 20, 5, 3000
    i64 = lambda lo, hi, n: rng.integers(lo, hi, n).astype(np.int64)
    emp = {"employee_id": rng.permutation(ne).astype(np.int64), "job_id": i64(0, nj + 5, ne),
           "manager_id": i64(-5, ne, ne), "department_id": i64(0, nd + 10, ne), "hire_date": i64(5000, 20000, ne),
           "commission_pct": rng.random(ne)}
    jobs = {"job_id": np.arange(nj, dtype=np.int64)}
    dept = {"department_id": np.arange(nd, dtype=np.int64), "manager_id": i64(0, ne + 100, nd),
            "location_id": i64(0, nl + 5, nd)}
    loc = {"location_id": np.arange(nl, dtype=np.int64), "country_id": i64(0, nc + 3, nl)}
    ctry = {"country_id": np.arange(nc, dtype=np.int64), "region_id": i64(0, nr + 1, nc)}
    reg = {"region_id": np.arange(nr, dtype=np.int64)}
    hist = {"employee_id": i64(0, ne + 500, nh), "job_id": i64(0, nj + 10, nh), "department_id": i64(0, nd + 5, nh),
            "level": i64(0, 16, nh), "offset": i64(0, 3, nh), "n": i64(-9, 9, nh), "k": i64(0, 5, nh)}
    chain = [("j", jobs), ("m", emp), ("d", dept), ("dm", emp), ("l", loc), ("c", ctry), ("r", reg), ("jh", hist),
             ("jj", jobs), ("dd", dept)]
    got = ex.sql(FIXTURE10_NUMERIC, on_dev(ex, emp), right=[on_dev(ex, t) for _, t in chain])
    # pandas: every table's columns prefixed by its alias
    pre = lambda a, t: pd.DataFrame({f"{a}.{k}": v for k, v in t.items()})
    m = pre("e", emp).merge(pre("j", jobs), left_on="e.job_id", right_on="j.job_id")
    for a, t, lk, rk in [("m", emp, "e.manager_id", "m.employee_id"), ("d", dept, "e.department_id", "d.department_id"),
                         ("dm", emp, "d.manager_id", "dm.employee_id"), ("l", loc, "d.location_id", "l.location_id"),
                         ("c", ctry, "l.country_id", "c.country_id"), ("r", reg, "c.region_id", "r.region_id"),
                         ("jh", hist, "e.employee_id", "jh.employee_id"), ("jj", jobs, "jh.job_id", "jj.job_id"),
                         ("dd", dept, "jh.department_id", "dd.department_id")]:
        m = m.merge(pre(a, t), left_on=lk, right_on=rk, how="left")
    assert got["Employee #"].tolist() == sorted(m["e.employee_id"].tolist())
    nn = lambda s: np.where(s.isna(), NULL, s.fillna(0)).astype(np.int64)
    lv, off = nn(m["jh.level"]), nn(m["jh.offset"])
    sh = lv >> np.clip(off, 0, 63)
    level = np.where(sh == 1, 1, np.where(sh == 2, 2, np.where(sh == 3, 3, nn(m["jh.n"]) * (nn(m["jh.k"]) + 3))))
    level = np.where(m["jh.level"].isna(), NULL, level)
    want = rows_of([m["e.employee_id"].to_numpy(), date_part(m["e.hire_date"].to_numpy(), 7),
                    m["e.commission_pct"].to_numpy(), nn(m["jh.job_id"]), level, nn(m["r.region_id"]),
                    nn(m["dd.location_id"])])
    cols = ["Employee #", "Hire Date", "Comission %", "History Job ID", "level", "region", "hist_location"]
    assert rows_of([filled(got[c]) for c in cols]) == want
    for c, src in (("History Job ID", "jh.job_id"), ("region", "r.region_id"), ("hist_location", "dd.location_id")):
        assert int(np.ma.getmaskarray(got[c]).sum()) == int(m[src].isna().sum()) > 0, c


def test_chain_step_types(ex):
    """RIGHT / FULL OUTER and LEFT SEMI / ANTI steps inside join chains (nut_plan_executen):
    RIGHT keeps every row of its table and NULL-extends every earlier one, FULL both; SEMI /
    ANTI filter the accumulated rows by a match (a NULL key has none).  pandas merges."""
    rng = np.random.default_rng(55)
    na, nb, nc = 3000, 2500, 800
    A = {"a_k": rng.integers(0, 2000, na).astype(np.int64), "a_v": rng.integers(-100, 100, na).astype(np.int64)}
    B = {"b_k": rng.permutation(2500).astype(np.int64), "b_x": rng.integers(0, 1200, nb).astype(np.int64)}
    C = {"c_k": rng.permutation(1000)[:nc].astype(np.int64), "c_v": rng.integers(0, 10**6, nc).astype(np.int64)}
    dA, dB, dC = pd.DataFrame(A), pd.DataFrame(B), pd.DataFrame(C)
    ab = dA.merge(dB, left_on="a_k", right_on="b_k")
    tabs = [on_dev(ex, B), on_dev(ex, C)]
    cols = ("a_k", "a_v", "b_x", "c_k", "c_v")
    nn = lambda s: np.where(s.isna(), NULL, s.fillna(0)).astype(np.int64)
    for kw, how in (("right join", "right"), ("full outer join", "outer")):
        m = ab.merge(dC, left_on="b_x", right_on="c_k", how=how)
        got = ex.sql(f"select a_k, a_v, b_x, c_k, c_v from a join b on a_k = b_k {kw} c on b_x = c_k",
                     on_dev(ex, A), right=tabs)
        assert rows_of([filled(got[c]) for c in cols]) == rows_of([nn(m[c]) for c in cols]), how
        got = ex.sql(f"select count(*) as n, count(a_v) as ca, sum(a_v) as sa, count(c_v) as cc, sum(c_v) as sc "
                     f"from a join b on a_k = b_k {kw} c on b_x = c_k", on_dev(ex, A), right=tabs)
        assert [got[k][0] for k in ("n", "ca", "sa", "cc", "sc")] == [
            len(m), int(m.a_v.notna().sum()), int(m.a_v.sum()), int(m.c_v.notna().sum()), int(m.c_v.sum())], how
    for kw, keep in (("left semi join", True), ("left anti join", False)):
        m = ab[ab.b_x.isin(dC.c_k) == keep]
        got = ex.sql(f"select a_k, a_v, b_x from a join b on a_k = b_k {kw} c on b_x = c_k", on_dev(ex, A), right=tabs)
        assert rows_of([got[c] for c in ("a_k", "a_v", "b_x")]) == rows_of([m[c].to_numpy() for c in ("a_k", "a_v", "b_x")])
    # after LEFT, a NULL-extended ON key: ANTI keeps those rows, SEMI drops them
    ab_l = dA.merge(dB, left_on="a_k", right_on="b_k", how="left")
    for kw, keep in (("left semi join", True), ("left anti join", False)):
        m = ab_l[ab_l.b_x.isin(dC.c_k) == keep]
        got = ex.sql(f"select a_k, a_v, count(*) as n from a left join b on a_k = b_k {kw} c on b_x = c_k "
                     "group by a_k, a_v", on_dev(ex, A), right=tabs)
        g = m.groupby(["a_k", "a_v"]).size()
        assert rows_of([got["a_k"], got["a_v"], got["n"]]) == sorted((k[0], k[1], int(v)) for k, v in g.items()), kw
    # RIGHT then LEFT through a key of the NULL-extended table
    m = dA.merge(dB, left_on="a_k", right_on="b_k", how="right").merge(dC, left_on="a_v", right_on="c_k", how="left")
    got = ex.sql("select b_k, a_v, c_v from a right join b on a_k = b_k left join c on a_v = c_k", on_dev(ex, A),
                 right=tabs)
    assert rows_of([filled(got[c]) for c in ("b_k", "a_v", "c_v")]) == rows_of([nn(m[c]) for c in ("b_k", "a_v", "c_v")])
    from nutdb_amd import NutError
    with pytest.raises(NutError, match="are not output"):
        ex.sql("select c_v from a join b on a_k = b_k left semi join c on b_x = c_k", on_dev(ex, A), right=tabs)
