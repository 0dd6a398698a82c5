#!/usr/bin/env python3
"""nutexec benchmark — BASELINE.json metric:
   "rows/sec filter->group-by on 1e9-row i64/f64; achieved HBM GB/s vs peak"

Default workload (N=1): BASELINE config 4, the TPC-H Q1-shape filter -> group-by
  SELECT l_returnflag, l_linestatus, sum(l_quantity), sum(l_extendedprice),
         sum(l_extendedprice*(1-l_discount)), count(*)
  FROM lineitem WHERE l_shipdate <= 10471 GROUP BY l_returnflag, l_linestatus
on 1e9 rows per GPU (6 x 8 B columns = 48 GB resident in HBM).  With --gpus N
(torchrun, one rank per GPU) every rank scans its own 1e9-row shard (weak scaling)
through the library's own multi-GPU path, nut_dist_* in libnutexec.so (what a Rust
host binds): ncclCommInitRank per process, local pre-aggregation,
partial groups exchanged by key hash with one RCCL all-to-all, owner merge, gather to
rank 0.  torch.distributed (gloo, CPU) is only the control plane: it broadcasts the
RCCL unique id and provides the barriers and the max-over-ranks time.

A "step" = one complete query over the resident columns (kernels + exchange + result
to host).  Other configs: --workload groupby (config 3), filter (config 2), sort
(config 5), q12expr (expression mode), join (SURVEY.md §8(f)4 hash join).

Prints ONE JSON line on rank 0 (contract in the task statement), with
  roofline     — the dominant kernel's algorithmic bytes / its mean device time
                 (hipEvents on the launch stream, via nut_ctx_kernel_time)
  cpu_baseline — the C oracle (oracle/, OpenMP over the host cores) on a bounded
                 sample of the same workload, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "rows/sec filter->group-by on 1e9-row i64/f64; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", default="q1", choices=["q1", "groupby", "filter", "scanexpr", "sort", "q12expr", "join", "q12join",
                                                   "parse"])
    p.add_argument("--rows", type=float, default=None, help="rows per GPU (default: config size)")
    p.add_argument("--groups", type=int, default=1000, help="groupby: distinct keys")
    p.add_argument("--skew", action="store_true",
                   help="groupby: Zipf-like keys from the same pool (pool index i on ~1/i of the rows)")
    p.add_argument("--selectivity", type=float, default=0.5, help="filter: fraction selected")
    p.add_argument("--key-range", type=float, default=None, metavar="FRACTION",
                   help="sort: keys uniform over this fraction of the int64 range (a sample-sort rank's share)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-copy-floor", action="store_true", help="skip the in-run device-copy floor probe")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    p.add_argument("--dist", action="store_true",
                   help="run N=1 through nut_dist_* too (one RCCL rank), as the N>1 runs do")
    p.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                   help="nut_ctx_set_option for A/B runs (Executor.OPTIONS names); recorded in config")
    return p.parse_args()


# ------------------------------------------------------------------ workloads
class Q1:
    name = "tpch_q1_shape_filter_groupby"
    cols_bytes = 48

    def __init__(self, ex, rows, row0):
        from nutdb_amd.workloads import Q1_COLS, Q1_DATE_K, gen
        self.ex = ex
        self.k = Q1_DATE_K
        self.cols = [gen(ex, spec, rows, row0=row0) for spec in Q1_COLS]
        self.rows = rows

    def local(self):
        return self.ex.q1(*self.cols, date_k=self.k)

    def run(self):  # single GPU step: the query and its (<= 6-group) result on the host
        g = self.local()
        r = g.to_host_words()
        g.free()
        return r

    @staticmethod
    def parity(gpu, cpu):
        (gk, gw), (ck, cw) = gpu, cpu
        return _cmp_groups(gk, gw, ck, cw, f64_cols=(0, 1, 2), rtol=1e-12)

    def run_dist(self, nd):  # N > 1: nut_dist_groupby of the same query (nut_q1's spec)
        from nutdb_amd import Agg, AggQuery
        sd, rf, ls, qty, price, disc = self.cols
        q = AggQuery(keys=[rf, ls], values=[qty, price, disc], preds=[(sd, "<=", self.k)],
                     aggs=[Agg("sum", "col", (0,)), Agg("sum", "col", (1,)), Agg("sum", "mul_1m", (1, 2)),
                           Agg("count")])
        g = nd.groupby([q], group_hint=8)[0]
        if g is None:
            return None
        r = g.to_host_words()
        g.free()
        return r

    kernel_kind = 1
    groups_hint = 8

    def config(self):
        return {"workload": self.name, "query": "TPC-H Q1 shape: WHERE l_shipdate <= 10471, GROUP BY "
                "l_returnflag, l_linestatus, 3 x SUM(f64) + COUNT(*)", "columns": "6 x 8 B (i64/f64)",
                "groups": 6, "selectivity": 0.973, "bytes_per_row": 48}


class GroupBy:
    name = "groupby_i64_sum_f64"
    cols_bytes = 16
    kernel_kind = 1

    def __init__(self, ex, rows, row0, groups, skew=False):
        from nutdb_amd.workloads import groupby_cols, gen
        self.ex = ex
        self.G = groups
        self.skew = skew
        self.groups_hint = groups
        self.key, self.val = [gen(ex, spec, rows, row0=row0) for spec in groupby_cols(groups, dyadic=True, skew=skew)]
        self.rows = rows
        self.out = None

    def local(self):
        from nutdb_amd import Agg, AggQuery
        return self.ex.groupby(AggQuery(keys=[self.key], values=[self.val], aggs=[Agg("sum", "col", (0,))]),
                               group_hint=self.G)

    def run(self):
        # one call, query -> ordered host result (nut_groupby_to_host: at large G the
        # key-range partitioned path, its transfer overlapped with the work)
        from nutdb_amd import Agg, AggQuery
        if self.out is None:
            # the result's host buffers: page-locked, allocated once and refilled every step
            # (fresh pageable arrays cost ~10 ms of first-touch page faults at 1e7 groups)
            rows = max(2 * self.G, 1024)
            self.out = tuple(torch.empty((rows, 1), dtype=torch.int64, pin_memory=True).numpy() for _ in range(2))
            self.q = AggQuery(keys=[self.key], values=[self.val], aggs=[Agg("sum", "col", (0,))])
        # views of the reused buffers: the last step's result stays
        return self.ex.groupby_to_host(self.q, group_hint=self.G, out=self.out)

    @staticmethod
    def parity(gpu, cpu):  # dyadic values: the f64 sums are exact, so compare bits
        (gk, gw), (ck, cw) = gpu, cpu
        return _cmp_groups(gk, gw, ck, cw, f64_cols=(), rtol=0.0)

    def run_dist(self, nd):  # N > 1: nut_dist_groupby; rank 0 receives the global groups
        from nutdb_amd import Agg, AggQuery
        g = nd.groupby([AggQuery(keys=[self.key], values=[self.val], aggs=[Agg("sum", "col", (0,))])],
                       group_hint=self.G)[0]
        if g is None:
            return None
        r = g.to_host_words()
        g.free()
        return r

    def config(self):
        return {"workload": self.name, "query": "SELECT key, SUM(val) FROM t GROUP BY key", "groups": self.G,
                "keys": "Zipf-like (GEN_SKEW_KEY, pool index i on ~1/i of the rows)" if self.skew
                else "uniform over the pool", "columns": "i64 key + f64 val (dyadic)", "bytes_per_row": 16}


class Filter:
    name = "filter_i64_compaction"
    kernel_kind = 0

    def __init__(self, ex, rows, row0, sel):
        from nutdb_amd.workloads import FILTER_COL, filter_k, gen
        self.ex = ex
        self.col = gen(ex, FILTER_COL, rows, row0=row0)
        self.k = filter_k(sel)
        self.sel = sel
        self.out = torch.empty(rows, dtype=torch.int64, device=ex.device)
        self.out_n = torch.zeros(1, dtype=torch.int64, device=ex.device)
        self.rows = rows
        self.cols_bytes = 8 + 8 * sel
        self.write_bytes = 8 * sel  # per row, of cols_bytes (the copy floor's write share)

    def run(self):
        self.ex.filter_i64_async(self.col, "<", self.k, self.out, self.out_n)
        return self.out, self.out_n

    def run_dist(self, nd):  # N > 1: shards are independent; one all-gather of counts
        return nd.filter_i64([self.col], "<", self.k)[0]

    @staticmethod
    def parity(gpu, cpu):
        out, out_n = gpu
        return _cmp_arrays(out[: int(out_n.item())].cpu().numpy(), cpu)

    def config(self):
        return {"workload": self.name, "query": "SELECT col FROM t WHERE col < k", "selectivity": self.sel,
                "bytes_per_row": 8 + 8 * self.sel}


class ScanExpr:
    """Expression-mode scan: SELECT a FROM t WHERE a < b over two int64
    columns (selectivity 0.5): nut_select_rows (WHERE compiled per query, row ids in row
    order) + the gather of `a` through the ids.  Roofline on the scan kernel: 16 B read +
    8 B per selected row id written."""
    name = "scan_expr_i64_compaction"
    kernel_kind = 0

    def __init__(self, ex, rows, row0):
        self.ex = ex
        self.a = ex.gen_column(1, 0x81, rows, row0=row0)
        self.b = ex.gen_column(1, 0x82, rows, row0=row0)
        self.where = [("col", 0), ("col", 1), ("lt",)]
        self.rows = rows
        self.cols_bytes = 16 + 8 * 0.5
        self.write_bytes = 8 * 0.5

    def run(self):  # results stay in HBM (as nut_plan_execute's scan results do)
        ids = self.ex.select_rows([self.a, self.b], self.where)
        return self.ex.gather(self.a, ids)

    @staticmethod
    def parity(gpu, cpu):
        return _cmp_arrays(gpu.cpu().numpy(), cpu)

    def config(self):
        return {"workload": self.name, "query": "SELECT a FROM t WHERE a < b (expression-mode scan)",
                "selectivity": 0.5, "bytes_per_row": self.cols_bytes,
                "step": "select kernel (row ids) + gather of a, results in HBM"}


class Sort:
    """config 5: ORDER BY a full-range i64 key.  N=1: local hybrid MSD radix sort
    (msd_sort.hip: two segmented scatter levels + on-chip local sorts for 1.25e9 random
    keys).  N>1: sample sort — splitters from an all_gather'd sample, local stable
    partition into skew-safe key ranges (nut_partition_i64), ONE RCCL all-to-all of keys,
    local sort of the received range (nut_dist_sort_i64).  Rank r ends with the r-th key
    range.  Algorithmic bytes come from the library (nut_ctx_sort_stats): 8 B/key per
    histogram read, 16 B/key per scatter level, local sort and copy."""
    name = "sort_i64_radix"
    kernel_kind = 2

    def __init__(self, ex, rows, row0, world=1, key_range=None):
        from nutdb_amd.workloads import gen, sort_col
        self.ex = ex
        self.key_range = key_range
        self.col = gen(ex, sort_col(key_range), rows, row0=row0)
        self.out = torch.empty_like(self.col) if world == 1 else None
        self.rows = rows
        self.world = world
        self.sort_bytes, self.levels = 0, 0

    # roofline numerator: SURVEY.md §8(d)'s HBM lower bound, one read + one write of every
    # key (16 B/key); the bytes the passes actually stream are reported beside it
    cols_bytes = 16
    write_bytes = 8  # copy floor: one read and one write of every key

    @property
    def pass_bytes(self):
        # per row of this rank's shard; N>1 adds the partition (8 B histogram + 16 B pass)
        return self.sort_bytes / self.rows + (24 if self.world > 1 else 0)

    def run(self):
        self.ex.sort_i64(self.col, out=self.out)
        self.sort_bytes, self.levels = self.ex.sort_stats()
        return self.out

    def run_dist(self, nd):  # the received range stays in the member's buffer (no copy)
        r = nd.sort_i64([self.col], copy=False)[0]
        self.sort_bytes, self.levels = nd.sort_stats()
        return r

    @staticmethod
    def parity(gpu, cpu):
        return _cmp_arrays(gpu.cpu().numpy(), cpu)

    def config(self):
        kr = "full-range i64" if self.key_range is None else f"i64 keys over {self.key_range:g} of the int64 range"
        return {"workload": self.name, "query": f"SELECT k FROM t ORDER BY k ({kr})",
                "algorithm": f"hybrid MSD radix: {self.levels} segmented scatter levels + on-chip local sorts"
                + ("; sample sort across ranks: partition by P-1 splitters + RCCL all-to-all" if self.world > 1
                   else ""),
                "bytes_per_row": self.cols_bytes, "roofline_bytes": "16 B/key HBM lower bound (SURVEY.md §8(d))",
                "pass_bytes_per_row": self.pass_bytes,
                "xgmi_bytes_per_row": 8.0 * (self.world - 1) / self.world}


class Q12Expr:
    """Expression mode: the reference fixture tests/sql/5.sql (TPC-H Q12
    shape, integer codes for its strings) through SQL -> plan -> a kernel compiled for
    the query.  Column-vs-column predicates, IN, CASE inside SUM.  Single GPU."""
    name = "q12_shape_expression_groupby"
    cols_bytes = 56
    kernel_kind = 1

    def __init__(self, ex, rows, row0):
        from nutdb_amd.sql import Plan
        from nutdb_amd.workloads import Q12_COLS, Q12_SQL, gen
        self.ex = ex
        self.cols = {spec[0]: gen(ex, spec, rows, row0=row0) for spec in Q12_COLS}
        self.plan = Plan(Q12_SQL)
        self.rows = rows

    def run(self):
        return self.plan.execute(self.ex, self.cols, group_hint=8)

    @staticmethod
    def parity(gpu, cpu):
        ck, cw = cpu[0], cpu[1]
        return _cmp_groups(np.stack([gpu["l_shipmode"]], 1), np.stack([gpu["high_line_count"],
                           gpu["low_line_count"]], 1).view(np.uint64), ck, cw, f64_cols=(), rtol=0.0)

    def config(self):
        return {"workload": self.name, "query": "reference tests/sql/5.sql (TPC-H Q12 shape; integer codes for "
                "its strings): 4 column-vs-column / IN predicates, 2 x SUM(CASE ...), GROUP BY l_shipmode",
                "columns": "7 x 8 B (i64)", "groups": 2, "bytes_per_row": 56,
                "kernel": "expression mode (hipRTC-compiled per query shape)"}


class Join:
    """INNER hash equi-join on int64 keys, TPC-H orders x lineitem shape —
    `rows` probe keys (lineitem.l_orderkey) against rows/4 unique build keys
    (orders.o_orderkey), 90 % of probe rows matching one build row.  One step = build
    (bucket count, scan, fill) + probe count + probe write of (probe_idx, build_idx) pairs
    in probe-row order (join.hip).  Algorithmic bytes: build keys read once (8 B) and the
    CSR table written once (16 B) per build row; probe keys read once (8 B) per probe row;
    16 B per output pair.  The table's random reads (bucket offsets, keys, rows) are not
    algorithmic bytes: they show up in the PMC traffic."""
    name = "join_i64_hash"
    kernel_kind = 3
    write_bytes = None  # random-read bound (§4.4): a streaming copy floor does not apply

    def __init__(self, ex, rows, row0, world=1, rank=0):
        self.ex = ex
        self.rows = rows
        self.nb = rows // 4
        self.world, self.rank = world, rank
        self.build = ex.gen_column(0, 0x71 + row0, self.nb)  # 62-bit: unique w.h.p.
        sel = ex.gen_column(0, 0x72 + row0, rows)
        self.probe = torch.where(sel % 10 == 0, sel | (1 << 62), self.build[sel % self.nb])
        del sel
        self.npairs = 0

    @property
    def cols_bytes(self):  # per probe row, of the join kernels the roofline times (N>1: local join)
        return (24.0 * self.nb + 8.0 * self.rows + 16.0 * self.npairs) / self.rows

    def run(self):
        pi, bi = self.ex.join_i64(self.build, self.probe, "inner")
        self.npairs = pi.numel()
        return pi, bi

    def run_dist(self, nd):  # global row ids; pairs stay in the member's buffers
        r = nd.join_i64([self.build], [self.probe], "inner", [self.rank * self.nb], [self.rank * self.rows],
                        copy=False)[0]
        self.npairs = int(r[2])
        return r

    @staticmethod
    def parity(gpu, cpu):
        # build keys are unique w.h.p., but the ABI leaves the build rows of one probe row
        # unordered: compare the pair sets ordered by (probe row, build row)
        g = [t.cpu().numpy() for t in gpu]
        og, oc = np.lexsort((g[1], g[0])), np.lexsort((cpu[1], cpu[0]))
        r = _cmp_arrays(g[0][og], cpu[0][oc])
        return r if not r["ok"] else _cmp_arrays(g[1][og], cpu[1][oc])

    def config(self):
        return {"workload": self.name, "query": "SELECT ... FROM lineitem JOIN orders ON l_orderkey = o_orderkey "
                "(join index: probe_idx, build_idx)", "build_rows": self.nb, "probe_rows": self.rows,
                "pairs": self.npairs, "match_rate": 0.9, "bytes_per_row": self.cols_bytes,
                "unit_rows": "probe rows",
                "algorithm": "open-addressing hash join, one ordered probe pass" + (
                    "; both sides hash-partitioned by key owner + one RCCL all-to-all each, local joins"
                    if self.world > 1 else ""),
                "xgmi_bytes_per_row": 16.0 * (1 + self.nb / self.rows) * (self.world - 1) / self.world,
                "partition_bytes_per_row": 48.0 * (1 + self.nb / self.rows) if self.world > 1 else 0.0}


Q12J_SQL = """select l_shipmode,
    sum(case when o_orderpriority = 1 or o_orderpriority = 2 then 1 else 0 end) as high_line_count,
    sum(case when o_orderpriority <> 1 and o_orderpriority <> 2 then 1 else 0 end) as low_line_count
  from orders join lineitem on o_orderkey = l_orderkey
  where l_shipmode in (3, 5) and l_commitdate < l_receiptdate and l_shipdate < l_commitdate
  group by l_shipmode order by l_shipmode"""


def q12j_tables(gen_i, rows):
    """orders (rows/4 unique keys, priority 1..5) and lineitem (rows, every line on an
    order; ship mode 0..6, three dates in [8000, 10000)) from a column generator
    gen_i(kind, seed, n, a, b) (device or oracle)."""
    no = max(rows // 4, 1)
    okey = gen_i(0, 0x91, no, 0, 0)
    orders = {"o_orderkey": okey, "o_orderpriority": gen_i(5, 0x92, no, 1, 5)}
    sel = gen_i(0, 0x93, rows, 0, 0) % no
    lineitem = {"l_orderkey": okey[sel], "l_shipmode": gen_i(5, 0x94, rows, 0, 7),
                "l_shipdate": gen_i(5, 0x95, rows, 8000, 2000), "l_commitdate": gen_i(5, 0x96, rows, 8000, 2000),
                "l_receiptdate": gen_i(5, 0x97, rows, 8000, 2000)}
    return orders, lineitem


class Q12Join:
    """TPC-H Q12 as written — orders JOIN lineitem ON o_orderkey = l_orderkey — through
    SQL -> plan -> nut_plan_execute2: the lineitem-only WHERE conjuncts are pushed below the
    join (expression-mode scan of lineitem, ~4.8 % selected), the join runs on the selected
    lines against all orders, the priority is gathered through the join index and the
    CASE sums run in the expression-mode group-by.  Roofline on the pushed-down scan kernel
    (4 x 8 B lineitem columns read + 8 B per selected id)."""
    name = "tpch_q12_join"
    kernel_kind = 0

    def __init__(self, ex, rows, row0):
        from nutdb_amd.sql import Plan
        self.ex = ex
        self.rows = rows
        self.orders, self.lineitem = q12j_tables(
            lambda k, seed, n, a, b: ex.gen_column(k, seed, n, a=a, b=b), rows)
        self.plan = Plan(Q12J_SQL)
        self.cols_bytes = 32 + 8 * (2 / 7) / 6
        self.write_bytes = self.cols_bytes - 32

    def run(self):
        return self.plan.execute_join(self.ex, self.orders, self.lineitem, group_hint=8)

    @staticmethod
    def parity(gpu, cpu):
        got = [(int(m), int(h), int(lo)) for m, h, lo in zip(gpu["l_shipmode"], gpu["high_line_count"],
                                                              gpu["low_line_count"])]
        want = [r for r in cpu if r[1] + r[2] > 0]
        return {"ok": got == want, "rows": len(got)} if got == want else {"ok": False, "got": got, "want": want}

    def config(self):
        return {"workload": self.name, "query": "TPC-H Q12 (integer codes for ship mode / priority): orders JOIN "
                "lineitem, IN + 2 date comparisons, 2 x SUM(CASE ...) GROUP BY l_shipmode",
                "lineitem_rows": self.rows, "orders_rows": self.rows // 4, "bytes_per_row": self.cols_bytes,
                "plan": "WHERE pushed below the join (select kernel) -> hash join (selected lines x orders) -> "
                        "gathers -> expression-mode group-by"}


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline(args, workload: str, target_s: float):
    """The C oracle on the host cores, same synthetic workload.  Columns are generated
    once (not timed); the scan is timed repeatedly up to ~target_s and the best run is
    reported."""
    from oracle import oracle as orc
    from nutdb_amd.workloads import FILTER_COL, Q1_COLS, Q1_DATE_K, filter_k, groupby_cols, sort_col
    threads = orc.max_threads()

    def prepare(n):
        if workload == "q1":
            sd, rf, ls, qty, price, disc = [orc.gen(s, n) for s in Q1_COLS]
            return lambda: orc.groupby([rf, ls], [(0, 0, (0,)), (0, 0, (1,)), (0, 4, (1, 2)), (1, 0, ())],
                                       values=[qty, price, disc], preds=[(sd, 1, Q1_DATE_K)], cap=64)
        if workload == "groupby":
            key, val = [orc.gen(s, n) for s in groupby_cols(args.groups, dyadic=True, skew=args.skew)]
            return lambda: orc.groupby([key], [(0, 0, (0,))], values=[val], cap=max(args.groups, 1))
        if workload == "sort":
            col = orc.gen(sort_col(args.key_range), n)
            return lambda: orc.sort_i64(col)
        if workload == "q12join":
            o, li = q12j_tables(lambda k, seed, m, a, b: orc.gen_column(k, seed, m, a=a, b=b), n)

            lcols = [li["l_shipmode"], li["l_commitdate"], li["l_receiptdate"], li["l_shipdate"]]
            where = [("col", 0), ("i64", 0, 3), ("eq",), ("col", 0), ("i64", 0, 5), ("eq",), ("or",), ("col", 1),
                     ("col", 2), ("lt",), ("and",), ("col", 3), ("col", 1), ("lt",), ("and",)]

            def q12():  # the pushed-down WHERE in C on every core (orc_eval_int), then the join
                ids = np.flatnonzero(orc.eval_int(where, lcols, n))
                pi, bi = orc.join_i64_c(o["o_orderkey"], li["l_orderkey"][ids], "inner")
                pr, mode = o["o_orderpriority"][bi], li["l_shipmode"][ids[pi]]
                hi = (pr == 1) | (pr == 2)
                return [(s_, int(np.sum(hi & (mode == s_))), int(np.sum(~hi & (mode == s_)))) for s_ in (3, 5)]
            return q12
        if workload == "scanexpr":  # the WHERE program in C on every core, numpy compaction
            a, b = orc.gen_column(1, 0x81, n), orc.gen_column(1, 0x82, n)
            return lambda: a[orc.eval_int([("col", 0), ("col", 1), ("lt",)], [a, b], n) != 0]
        if workload == "join":  # the columns of bench's Join (same generator, rank 0)
            nb = n // 4
            b = orc.gen_column(0, 0x71, nb)
            sel = orc.gen_column(0, 0x72, n)
            p = np.where(sel % 10 == 0, sel | (1 << 62), b[sel % max(nb, 1)])
            del sel
            return lambda: orc.join_i64_c(b, p, "inner")
        if workload == "q12expr":
            from nutdb_amd.workloads import Q12_AGGS, Q12_COLS, Q12_WHERE
            from oracle.expr import groupby_prog
            cols = [orc.gen(s, n) for s in Q12_COLS]
            return lambda: groupby_prog([cols[2]], cols, Q12_WHERE, Q12_AGGS, threads=threads, engine="c")
        col = orc.gen(FILTER_COL, n)
        k = filter_k(args.selectivity)
        return lambda: orc.filter_i64(col, 0, k)

    last = [None]

    def timed(fn):
        last[0] = None
        t0 = time.perf_counter()
        last[0] = fn()
        return time.perf_counter() - t0

    full =int(args.rows) if args.rows else {"q1": 10**9, "groupby": 10**9, "filter": 10**8,
                                             "sort": 1_250_000_000, "q12expr": 10**9, "join": 10**9,
                                             "scanexpr": 10**8, "q12join": 10**9}[workload]
    probe = min(full, 4_000_000)
    per_row = timed(prepare(probe)) / probe
    sample = int(min(full, max(probe, target_s / max(per_row, 1e-12))))
    if workload == "join":  # the pair-set parity check sorts every pair on the host: keep it to seconds
        sample = min(sample, 50_000_000)
    fn = prepare(sample)
    times = [timed(fn)]
    while sum(times) < target_s and len(times) < 10:
        times.append(timed(fn))
    dt = min(times)
    if workload == "join":
        how, cores = (f"C hash join (oracle/oracle.c orc_join_i64: CSR bucket table + two-pass probe), OpenMP "
                      f"over {threads} host threads; probe rows, build = probe/4"), threads
    elif workload == "scanexpr":
        how, cores = (f"C expression evaluator (oracle/oracle.c orc_eval_int, OpenMP over {threads} host threads) + "
                      f"numpy boolean compaction (1 thread)"), threads
    elif workload == "q12join":
        how, cores = (f"C expression evaluator for the pushed-down WHERE + C hash join (oracle/oracle.c, OpenMP over "
                      f"{threads} threads) + numpy CASE sums"), threads
    elif workload == "q12expr":
        how, cores = (f"C expression evaluator (oracle/oracle.c orc_eval_int) + C oracle group-by, OpenMP over "
                      f"{threads} host threads"), threads
    elif workload == "groupby":
        how, cores = (f"C oracle (oracle/oracle.c orc_groupby: per-thread tables for few groups, key-range "
                      f"partitioned per-partition merge for many), OpenMP over {threads} host threads"), threads
    else:
        how, cores = f"C oracle (oracle/oracle.c), OpenMP over {threads} host threads", threads
    del fn
    info = {"value": sample / dt, "unit": "rows/s", "cores": cores, "kind": "port",
            "sample": f"{sample:.3g} rows of the same synthetic workload ({sample / full:.2f} of one GPU's "
                      f"rows), {how}, generation excluded, best of {len(times)} timed runs = {dt:.3f} s"}
    return info, last[0], sample


def _cmp_arrays(got, want):
    if got.shape != want.shape:
        return {"ok": False, "why": f"length {got.shape} != {want.shape}"}
    bad = np.flatnonzero(got != want)
    if len(bad):
        i = int(bad[0])
        return {"ok": False, "why": f"{len(bad)} mismatches, first at {i}: {got[i]} != {want[i]}"}
    return {"ok": True, "compare": "bit-exact"}


def _cmp_groups(gk, gw, ck, cw, f64_cols, rtol):
    """Group results (keys [G, nk] int64, words [G, na] uint64, both ordered by key):
    keys and integer / count words bit-exact, f64 sum columns within rtol relative
    (rtol 0: bit-exact)."""
    if gk.shape != ck.shape or not np.array_equal(gk, ck):
        return {"ok": False, "why": f"group keys differ ({len(gk)} vs {len(ck)} groups)"}
    worst = 0.0
    for j in range(cw.shape[1]):
        if j in f64_cols and rtol > 0:
            a, b = gw[:, j].view(np.float64), cw[:, j].view(np.float64)
            err = float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if len(a) else 0.0
            worst = max(worst, err)
            if err > rtol:
                return {"ok": False, "why": f"aggregate {j}: rel err {err:.3g} > {rtol}"}
        elif not np.array_equal(gw[:, j], cw[:, j]):
            return {"ok": False, "why": f"aggregate {j} differs"}
    r = {"ok": True, "groups": int(len(gk)), "compare": "keys + integer aggregates bit-exact"}
    r["compare"] += f", f64 sums max rel err {worst:.2g} (tol {rtol})" if f64_cols and rtol > 0 else \
        ", f64 sums bit-exact"
    return r


# ------------------------------------------------------------------ main
def parse_bench(args):
    """BASELINE config 1: parse-only over the reference's SQL fixtures (tests/golden/sql:
    tests/sql/1..14.sql + the two criterion bench statements), CPU only, through the C ABI
    (nut_sql_parse + nut_stmt_free per statement; ctypes call overhead included)."""
    import ctypes as C
    from nutdb_amd._lib import lib
    files = sorted((ROOT / "tests" / "golden" / "sql").glob("*.sql"))
    stmts = [f.read_bytes() for f in files]
    iters = max(args.steps, 1) * 100
    h = C.c_void_p()
    for s in stmts * max(args.warmup, 1):
        assert lib.nut_sql_parse(s, len(s), C.byref(h)) == 0
        lib.nut_stmt_free(h)
    per = {}
    t_all = 0.0
    for f, s in zip(files, stmts):
        n = len(s)
        t0 = time.perf_counter()
        for _ in range(iters):
            lib.nut_sql_parse(s, n, C.byref(h))
            lib.nut_stmt_free(h)
        dt = time.perf_counter() - t0
        t_all += dt
        per[f.name] = round(dt / iters * 1e6, 3)
    total = iters * len(stmts)
    line = {
        "metric": "statements/sec parse-only over tests/sql fixtures (CPU)", "value": total / t_all,
        "unit": "statements/s", "n_gpus": 0, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": t_all * 1e3 / max(args.steps, 1), "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "utf8", "data": "reference fixtures (tests/golden/sql)",
        "config": {"workload": "parse", "statements": len(stmts), "iterations_each": iters,
                   "us_per_statement": per, "bytes_total": sum(len(s) for s in stmts),
                   "note": "single host thread; includes ctypes call overhead (~0.5 us/call)"},
        "roofline": None, "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)


def main():
    args = parse()
    if args.workload == "parse":
        parse_bench(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("bench.py: --gpus N>1 must be launched with torch.distributed.run", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local_rank)
    from nutdb_amd import Executor
    ex = Executor(local_rank)
    nd = None
    if world > 1 or args.dist:
        # control plane only (CPU): the RCCL unique id, barriers, the max-over-ranks time;
        # every data exchange runs inside libnutexec.so (nut_dist_*, ncclCommInitRank)
        if world == 1:  # --dist without torchrun
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("gloo")
        from nutdb_amd.dist import NutDist
        uid = [NutDist.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        nd = NutDist.create_rank(world, rank, uid[0], local_rank)
    options = {}
    for o in args.option:
        name, val = o.split("=", 1)
        ex.set_option(name, int(val))
        options[name] = int(val)
    default_rows = {"q1": 1e9, "groupby": 1e9, "filter": 1e8, "sort": 1.25e9, "q12expr": 1e9,
                    "join": 1e9, "scanexpr": 1e8, "q12join": 1e9}[args.workload]
    rows = int(args.rows or default_rows)
    row0 = rank * rows
    if args.workload in ("q12expr", "q12join") and world > 1:
        print(f"bench.py: {args.workload} is a single-GPU workload", file=sys.stderr)
        sys.exit(2)
    w = make_workload(args, ex, rows, row0, world, rank)
    torch.cuda.synchronize()
    last = [None]
    if nd is not None:
        for o in args.option:
            name, val = o.split("=", 1)
            from nutdb_amd._lib import lib
            lib.nut_ctx_set_option(nd.ctx(0), ex.OPTIONS[name], int(val))

    def step():
        last[0] = None  # the previous step's result is dropped before the next one runs
        last[0] = w.run() if nd is None else w.run_dist(nd)

    for _ in range(args.warmup):
        step()
    (ex if nd is None else nd).enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, launches = (ex if nd is None else nd).kernel_time(w.kernel_kind)
    (ex if nd is None else nd).enable_timing(False)
    gb_stats = ex.groupby_stats() if nd is None and args.workload in ("q1", "groupby", "q12expr", "q12join") else None
    if gb_stats is not None and gb_stats["path"] == "partitioned_ordered":
        gb_stats["overflow_rows"] = ex.groupby_overflow_rows()
        gb_stats["heavy_keys"], gb_stats["heavy_rows"] = ex.groupby_heavy()
    if nd is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed * 1e3 / args.steps
    total_rows = rows * world * args.steps
    value = total_rows / elapsed
    # per step: the step's algorithmic bytes over its device time in the hot kernels
    # (one launch per step except the multi-GPU merge / sample-sort partition)
    avg_kernel_ms = kern_ms / args.steps
    bytes_per_step = w.cols_bytes * rows
    achieved = bytes_per_step / (avg_kernel_ms * 1e-3) / 1e9 if launches else None
    # PMC-measured HBM traffic of the same kernel/config, if profiled (profiles/pmc_*.json)
    # (not measured in this run: rocprofv3 --pmc cannot run under the timed bench; the
    # source file, its commit and date travel with the number as traffic_source)
    traffic, traffic_src = None, None
    pmc = ROOT / "profiles" / f"pmc_{w.name}.json"
    if w.name == "groupby_i64_sum_f64":  # partitioned G: its own per-step file, if measured
        pg = ROOT / "profiles" / f"pmc_{w.name}_g{args.groups}{'_skew' if args.skew else ''}.json"
        pmc = pg if pg.exists() else pmc
    if pmc.exists():
        try:
            d = json.loads(pmc.read_text())
            if int(d.get("rows", -1)) == rows and (w.name != "groupby_i64_sum_f64" or (
                    int(d.get("groups", 1000)) == args.groups and bool(d.get("skew", False)) == bool(args.skew))):
                traffic = d.get("hbm_bytes_per_launch")
                m = d.get("measured", {})
                traffic_src = (f"profiles/{pmc.name}: {d.get('per', 'per launch')}, "
                               f"{d.get('correction', '')}; measured {m.get('date_utc', 'round 1')} at commit "
                               f"{m.get('commit', 'unknown')} (separate rocprofv3 --pmc passes of the same command)")
        except Exception:
            traffic = None
    # copy floor: the in-build streaming probe moving the same read / write
    # bytes as the timed kernels, on this board, right after the timed loop
    copy_floor = None
    wb = getattr(w, "write_bytes", 0)
    if rank == 0 and not args.no_copy_floor and wb is not None and launches:
        rb = int((w.cols_bytes - wb) * rows)
        probe_ms = ex.stream_probe(rb, int(wb * rows), reps=5)
        copy_floor = {"kernel": "nut_stream_probe (16-B non-temporal loads / stores, same read:write ratio, "
                                "best of 2 / 4 / 8 workgroups per CU x 5 launches)",
                      "read_bytes": rb, "write_bytes": int(wb * rows), "ms": probe_ms,
                      "achieved": bytes_per_step / (probe_ms * 1e-3) / 1e9,
                      "frac_of_peak": bytes_per_step / (probe_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "kernel_frac_of_copy": probe_ms / avg_kernel_ms}
    # the compiled Q1 kernel's launch shapes on this board (untimed, after the timed loop):
    # the shape the library's probe chose, and each candidate's kernel time over the same
    # full-size step (3 runs each, best), next to the copy floor above
    shapes = None
    if args.workload == "q1" and nd is None and rank == 0 and not args.no_copy_floor:
        shapes = {"chosen": ex.priv_shape(), "kernel_ms_full_size": {}}
        for bd, bl in ((192, 2), (128, 3), (128, 4)):
            old = ex.set_option("priv_bd", bd), ex.set_option("priv_blocks", bl)
            best = None
            for _ in range(3):
                ex.enable_timing(True)
                w.run()
                ms, n = ex.kernel_time(w.kernel_kind)
                ex.enable_timing(False)
                best = ms / max(n, 1) if best is None else min(best, ms / max(n, 1))
            ex.set_option("priv_bd", old[0])
            ex.set_option("priv_blocks", old[1])
            shapes["kernel_ms_full_size"][f"{bd}x{bl}"] = round(best, 4)
        if copy_floor:
            shapes["copy_floor_ms"] = copy_floor["ms"]
    parity = None
    cpu = None
    if rank == 0 and world == 1 and nd is None and not args.no_cpu_baseline:
        cpu, cpu_res, sample = cpu_baseline(args, args.workload, args.cpu_seconds)
        if args.workload == "groupby" and sample != rows:
            # full size: the pool keys are a bijection of an index, so the indexed dense-array
            # oracle checks the last timed step itself (exact, seconds at 1e9 rows x 1e7 groups)
            from oracle import oracle as orc
            from nutdb_amd.workloads import GB_KEY_SEED, GB_VAL_SEED
            del cpu_res
            t0 = time.perf_counter()
            ok, ow = orc.groupby_pool_dyadic(args.groups, rows, row0=0, key_seed=GB_KEY_SEED, val_seed=GB_VAL_SEED,
                                             kind=7 if args.skew else 2)
            cpu_res = (ok, np.ascontiguousarray(ow[:, :1]))
            sample = rows
            how = ("last timed step vs the indexed dense-array oracle (oracle.h orc_groupby_pool_dyadic, "
                   f"{time.perf_counter() - t0:.1f} s) on the same full-size input")
            gpu_res = last[0]
        elif sample == rows:
            how = "last timed step vs the CPU baseline's result on the same full-size input"
            gpu_res = last[0]
        else:  # the GPU rerun (untimed) on the CPU sample's input: the first `sample` rows
            how = f"GPU rerun (untimed) on the CPU sample's {sample} rows vs the CPU baseline's result"
            last[0] = None
            gpu_res = make_workload(args, ex, sample, 0, 1, 0).run()
        parity = {"rows": sample, "full_size": sample == rows, "method": how}
        if gb_stats is not None:
            parity["timed_path"] = gb_stats
            if sample != rows:
                parity["checked_path"] = ex.groupby_stats()
        parity.update(type(w).parity(gpu_res, cpu_res))
        del cpu_res, gpu_res
    if rank == 0:
        cfg = w.config()
        if gb_stats is not None:
            cfg["groupby_path"] = gb_stats
        if options:
            cfg["options"] = options
        if shapes is not None:
            cfg["launch_shape"] = shapes
        if nd is not None:
            cfg["dist"] = {"api": "nut_dist_create_rank + nut_dist_* (libnutexec.so, RCCL)", "nranks": nd.nranks,
                           "control_plane": "torch.distributed gloo (unique id, barriers, max time)"}
        cfg.update({"rows_per_gpu": rows, "parallelism": f"dp{world} (row shards; " + {
                        "q1": "key-hash all-to-all of partial groups", "groupby": "key-hash all-to-all of partial groups",
                        "sort": "sample sort: skew-safe key ranges + one all-to-all of keys",
                        "filter": "independent shards + all-gather of counts",
                        "join": "key-owner all-to-all of both sides"}.get(args.workload, "") + " over RCCL)"
                    if world > 1 else "single GPU", "gpu": ex.info()["name"],
                    "kernel_launches": launches, "kernel_ms_per_step": avg_kernel_ms})
        line = {
            "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "i64+f64", "data": "synthetic (counter-based splitmix64 columns "
            "generated in HBM)", "config": cfg,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         # the same bytes over the whole step's wall time (host overheads and any
                         # result copy included): reproducible from ms_per_step alone
                         "achieved_wall": bytes_per_step / (ms_step * 1e-3) / 1e9,
                         "frac_wall": bytes_per_step / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "copy_floor": copy_floor},
        }
        if cpu is not None:
            line["cpu_baseline"] = cpu
            line["parity"] = parity
        print(json.dumps(line), flush=True)
    if nd is not None:
        nd.close()
    ex.close()
    if nd is not None or world > 1:
        dist.destroy_process_group()
    if parity is not None and not parity["ok"]:
        print(f"bench.py: PARITY FAILURE vs the CPU oracle: {parity}", file=sys.stderr)
        sys.exit(1)


def make_workload(args, ex, rows, row0, world, rank):
    if args.workload == "q1":
        return Q1(ex, rows, row0)
    if args.workload == "groupby":
        return GroupBy(ex, rows, row0, args.groups, args.skew)
    if args.workload == "sort":
        return Sort(ex, rows, row0, world, args.key_range)
    if args.workload == "q12expr":
        return Q12Expr(ex, rows, row0)
    if args.workload == "join":
        return Join(ex, rows, row0, world, rank)
    if args.workload == "scanexpr":
        return ScanExpr(ex, rows, row0)
    if args.workload == "q12join":
        return Q12Join(ex, rows, row0)
    return Filter(ex, rows, row0, args.selectivity)


if __name__ == "__main__":
    main()
