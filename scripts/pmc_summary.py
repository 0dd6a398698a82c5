"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<tag>/) into one JSON: mean counter value
per dispatch for every kernel whose name contains one of the given substrings.
  python3 scripts/pmc_summary.py out.json "<what was run>" kernel_substr,... tag1 tag2 ..."""
import collections
import csv
import glob
import json
import subprocess
import sys

out, how, kernels, tags = sys.argv[1], sys.argv[2], sys.argv[3].split(","), sys.argv[4:]
res = collections.defaultdict(dict)
for tag in tags:
    for f in glob.glob(f"gpurun_out/pmc_{tag}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in kernels):
                acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            res[k][c] = {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
for k, cs in res.items():
    if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
        f = cs.get("FETCH_SIZE", {}).get("mean_per_dispatch", 0.0) * 1024 * 2  # KB, gfx950 wide-stream halving
        w = cs.get("WRITE_SIZE", {}).get("mean_per_dispatch", 0.0) * 1024
        cs["hbm_bytes_per_dispatch"] = {"read": f, "write": w, "total": f + w,
                                        "correction": "read = 2 x FETCH_SIZE KB, write = WRITE_SIZE KB"}
commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
json.dump({"how": how, "commit": commit, "kernels": res}, open(out, "w"), indent=1)
print(json.dumps({k: {c: round(v["mean_per_dispatch"]) if "mean_per_dispatch" in v else v for c, v in cs.items()}
                  for k, cs in res.items()}, indent=1)[:3000])
