"""Localise a fixture-9 (TPC-H Q22) mismatch: the substring WHERE alone, with the scalar
subquery, with the NOT EXISTS step, and the whole fixture, each against pandas."""
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from nutdb_amd import Executor  # noqa: E402
from nutdb_amd.table import Table  # noqa: E402

ex = Executor()
rng = np.random.default_rng(9)
nc, no = 20_000, 40_000
cc = rng.integers(10, 35, nc)
phone = np.array([f"{c}-{rng.integers(100, 999)}-{rng.integers(1000, 9999)}" for c in cc], dtype=object)
cust = {"c_custkey": rng.permutation(nc * 2)[:nc].astype(np.int64), "c_phone": phone,
        "c_acctbal": np.round(rng.uniform(-999.99, 9999.99, nc), 2)}
orders = {"o_custkey": rng.choice(cust["c_custkey"], no).astype(np.int64)}
t = Table(ex, "CREATE TABLE customer (c_custkey Int64, c_phone String, c_acctbal Float64)")
t.append(**cust)
o = Table(ex, "CREATE TABLE orders (o_custkey Int64)")
o.append(**orders)
d = pd.DataFrame(cust)
d["cc"] = d.c_phone.str[:2]
IN = "('13', '31', '23', '29', '30', '18', '17')"
codes = ["13", "31", "23", "29", "30", "18", "17"]
has = set(orders["o_custkey"])
avg = d.c_acctbal[(d.c_acctbal > 0) & d.cc.isin(codes)].mean()
cases = [
    ("in", f"select count(*) as n from customer where substring(c_phone, 1, 2) in {IN}", None,
     int(d.cc.isin(codes).sum())),
    ("in+sub", f"select count(*) as n from customer where substring(c_phone, 1, 2) in {IN} and c_acctbal > "
               f"(select avg(c_acctbal) from customer where c_acctbal > 0.00 and substring(c_phone, 1, 2) in {IN})",
     None, int((d.cc.isin(codes) & (d.c_acctbal > avg)).sum())),
    ("in+anti", f"select count(*) as n from customer where substring(c_phone, 1, 2) in {IN} and not exists "
                f"(select * from orders where o_custkey = c_custkey)", [o],
     int((d.cc.isin(codes) & ~d.c_custkey.isin(has)).sum())),
    ("all3", f"select count(*) as n from customer where substring(c_phone, 1, 2) in {IN} and c_acctbal > "
             f"(select avg(c_acctbal) from customer where c_acctbal > 0.00 and substring(c_phone, 1, 2) in {IN}) "
             f"and not exists (select * from orders where o_custkey = c_custkey)", [o],
     int((d.cc.isin(codes) & (d.c_acctbal > avg) & ~d.c_custkey.isin(has)).sum())),
    ("eq+anti", "select count(*) as n from customer where substring(c_phone, 1, 2) = '13' and not exists "
                "(select * from orders where o_custkey = c_custkey)", [o],
     int(((d.cc == "13") & ~d.c_custkey.isin(has)).sum())),
    ("col+anti", "select count(*) as n from customer where c_acctbal > 5000 and not exists "
                 "(select * from orders where o_custkey = c_custkey)", [o],
     int(((d.c_acctbal > 5000) & ~d.c_custkey.isin(has)).sum())),
]
for name, sql, joined, want in cases:
    try:
        got = t.sql(sql, joined=joined) if joined else t.sql(sql)
        print(f"{name:8s} got {int(got['n'][0])} want {want}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name:8s} error {e}", flush=True)
