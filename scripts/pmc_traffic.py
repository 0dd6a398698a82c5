#!/usr/bin/env python3
"""Turn a scripts/round_profile.sh directory into profiles/-ready summaries:
  summary.json       per-kernel trace stats (calls, avg ns) + per-dispatch PMC means
  pmc_<workload>.json HBM bytes per launch of the dominant kernel, read by bench.py
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is
exact for 16-B streaming stores and atomics (x 1024)."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from prof_summary import summarize  # noqa: E402

WORKLOAD_KERNEL = {"q1": ("tpch_q1_shape_filter_groupby", "agg_kernel"),
                   "groupby": ("groupby_i64_sum_f64", "agg_kernel"),
                   "filter": ("filter_i64_compaction", "filter_i64_staged_kernel"),
                   "sort": ("sort_i64_radix", "nut::ms_"),
                   "q12expr": ("q12_shape_expression_groupby", "agg_kernel"),
                   "join": ("join_i64_hash", "hj_"),
                   "scanexpr": ("scan_expr_i64_compaction", "select_kernel"),
                   "q12join": ("tpch_q12_join", "select_kernel")}
# sort: one step = every kernel of one MSD sort (2 histograms, 2 scatter levels, the
# local sort and its fallback); traffic is summed per step (one local-sort launch per step)
STEP_KERNEL = {"sort": "ms_local_kernel", "join": "hj_probe_kernel"}


def main():
    d = Path(sys.argv[1])
    args = sys.argv[2:]
    wl = args[args.index("--workload") + 1] if "--workload" in args else "q1"
    rows = float(args[args.index("--rows") + 1]) if "--rows" in args else {"q1": 1e9, "groupby": 1e9, "filter": 1e8,
                                                                           "sort": 1.25e9, "q12expr": 1e9,
                                                                           "join": 1e9, "scanexpr": 1e8,
                                                                           "q12join": 1e9}[wl]
    name, match = WORKLOAD_KERNEL[wl]
    groups = int(float(args[args.index("--groups") + 1])) if "--groups" in args else {"q1": 6, "groupby": 1000}.get(wl)
    step_kernel, exclude, fname = STEP_KERNEL.get(wl, ""), "", name
    per_desc = {"sort": "step (all ms_* kernels of one sort)", "join": "step (all hj_* kernels of one join)"}.get(
        wl, "launch of " + match)
    if wl == "groupby" and groups and groups >= 100000:
        # partitioned group-by: every library kernel of one step (scatter levels, heavy-key
        # pass, aggregation, ordering), column generation excluded; steps counted by a kernel
        # that runs once per step (the one capped level at G = 1e5, the range sample above)
        match, exclude = "nut::", "gen_column"
        step_kernel = "go_sample_kernel" if groups >= 1000000 else "gp_scatter_kernel"
        fname = f"{name}_g{groups}" + ("_skew" if "--skew" in args else "")
        per_desc = "step (all nut:: kernels of one group-by step except column generation)"
    s = summarize(d, match, step_kernel, exclude)
    c = s["counters"]
    traffic = None
    # join: the reads are dominated by random single-slot (64-B) requests, counted whole;
    # the x2 halving correction is for wide streaming reads only
    rmul = 1 if wl == "join" else 2
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        traffic = c["FETCH_SIZE"] * 1024 * rmul + c["WRITE_SIZE"] * 1024
    s["workload"] = name
    s["rows"] = int(rows)
    s["hbm_bytes_per_launch"] = traffic
    (d / "summary.json").write_text(json.dumps(s, indent=1))
    (d / f"pmc_{fname}.json").write_text(json.dumps({
        "workload": name, "rows": int(rows), "groups": groups, "skew": "--skew" in args,
        "kernel_match": match, "kernel_exclude": exclude or None, "hbm_bytes_per_launch": traffic,
        "dispatches": None if step_kernel else s.get("dispatches"),
        "fetch_size_kb": c.get("FETCH_SIZE"), "write_size_kb": c.get("WRITE_SIZE"),
        "per": per_desc,
        "measured": {"tag": d.name, "commit": os.environ.get("NUT_COMMIT", "unknown"),
                     "date_utc": time.strftime("%Y-%m-%dT%H:%MZ", time.gmtime()),
                     "how": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, one pass each, over bench.py "
                            + " ".join(args)},
        "correction": ("read = FETCH_SIZE (random 64-B slot reads dominate; the gfx950 x2 wide-stream "
                       "correction is not applied, so the ~12 GB of streaming key reads count half)"
                       if wl == "join" else "read = 2 x FETCH_SIZE (gfx950 wide-stream halving), write = WRITE_SIZE")},
        indent=1))
    print(json.dumps({"workload": name, "traffic": traffic, "kernels": s["kernels"][:3]}))


if __name__ == "__main__":
    main()
