cd "${GRAFT_REPO_ROOT}" || exit 1
for r in 1 2; do
  for t in 1024 512; do
    for g in 100000 10000000; do
      NUT_GP_T=$t timeout -k 10 200 python bench.py --workload groupby --groups $g --steps 6 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$r', 'T=$t', 'G=$g', 'kernel', round(d['config']['kernel_ms_per_step'], 3), 'step', round(d['ms_per_step'], 3), flush=True)" || exit 1
    done
    NUT_GP_T=$t timeout -k 10 200 python bench.py --workload join --steps 4 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$r', 'T=$t', 'join', 'kernel', round(d['config']['kernel_ms_per_step'], 3), flush=True)" || exit 1
  done
done
