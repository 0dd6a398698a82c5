#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory: per-kernel trace stats and the
PMC counters (mean per dispatch) of the kernels matching a name filter.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a
wide coalesced streaming read — reported both raw and x2."""
import collections
import csv
import glob
import json
import sys
from pathlib import Path


def summarize(d: Path, match: str = "agg_kernel", step_match: str = "", exclude: str = ""):
    out = {"kernels": [], "counters": {}}
    for f in glob.glob(str(d / "trace" / "*_kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            out["kernels"].append({"name": row["Name"][:100], "calls": int(row["Calls"]),
                                   "avg_ns": float(row["AverageNs"]), "pct": float(row["Percentage"])})
    for f in glob.glob(str(d / "*" / "*_counter_collection.csv")):
        # per dispatch (rows of one dispatch summed); the mean over the full-size dispatches
        # only — those within half of the largest — so a workload's smaller launches of the
        # same kernel (the Q1 launch-shape probe on 2^28 rows) do not dilute it
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for i, row in enumerate(csv.DictReader(open(f))):
            if match in row["Kernel_Name"] and not (exclude and exclude in row["Kernel_Name"]):
                per[row["Counter_Name"]][row.get("Dispatch_Id", i)] += float(row["Counter_Value"])
        for k, byd in per.items():
            v = list(byd.values())
            full = [x for x in v if x >= 0.5 * max(v)] if v else []
            if full:
                out["counters"][k] = sum(full) / len(full)
                out.setdefault("dispatches", {})[k] = {"kept": len(full), "of": len(v)}
    c = out["counters"]
    if step_match:
        # totals per step: every dispatch matching `match`, divided by the number of
        # dispatches of the once-per-step kernel `step_match`
        for f in glob.glob(str(d / "*" / "*_counter_collection.csv")):
            tot = collections.defaultdict(float)
            steps = collections.defaultdict(set)
            for row in csv.DictReader(open(f)):
                if match in row["Kernel_Name"] and not (exclude and exclude in row["Kernel_Name"]):
                    tot[row["Counter_Name"]] += float(row["Counter_Value"])
                if step_match in row["Kernel_Name"]:
                    steps[row["Counter_Name"]].add(row.get("Dispatch_Id", row.get("Correlation_Id", len(steps))))
            for k, v in tot.items():
                if steps[k]:
                    c[k] = v / len(steps[k])
    if "FETCH_SIZE" in c:
        c["HBM_READ_BYTES_x2corr"] = c["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in c:
        c["HBM_WRITE_BYTES"] = c["WRITE_SIZE"] * 1024
    return out


if __name__ == "__main__":
    d = Path(sys.argv[1])
    m = sys.argv[2] if len(sys.argv) > 2 else "agg_kernel"
    print(json.dumps(summarize(d, m), indent=1))
