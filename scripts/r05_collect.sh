#!/bin/bash
# copy one closing part's results (gpurun_out/r05/<name>/) into profiles/r05/final/<name>/
cd "$(dirname "$0")/.." || exit 1
for name in "$@"; do
  src=gpurun_out/r05/$name; dst=profiles/r05/final/$name
  mkdir -p "$dst"
  for f in bench.json bench.log kernel_stats.csv trace.log summary.json profile.log; do
    [ -f "$src/$f" ] && cp "$src/$f" "$dst/"
  done
  cp "$src"/pmc_*.json "$dst/" 2>/dev/null
  echo "$name: $(python3 -c "import json;d=json.load(open('$dst/bench.json'));print(round(d['ms_per_step'],3), round(d['config']['kernel_ms_per_step'],3))")"
done
