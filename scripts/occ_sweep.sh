#!/bin/bash
# Occupancy sweep of the compiled private-table kernels (Q1 / Q12 shapes) on ONE box, each
# run next to the in-run copy floor (nut_stream_probe) of the same bytes:
#   scripts/occ_sweep.sh <rounds> "<bd:blocks> ..." <bench args...>
# bd = threads per workgroup (NUT_OPT_PRIV_BD), blocks = workgroups per CU
# (NUT_OPT_PRIV_BLOCKS); 0:0 = the library default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
rounds=$1; cfgs=$2; shift 2
for round in $(seq 1 "$rounds"); do
  for cfg in $cfgs; do
    bd=${cfg%%:*}; bl=${cfg##*:}
    timeout -k 10 200 python bench.py "$@" --no-cpu-baseline --option priv_bd=$bd --option priv_blocks=$bl \
      2>/dev/null | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
r = d['roofline']; cf = r.get('copy_floor') or {}
k = d['config']['kernel_ms_per_step']
print('$round', 'bd=$bd blocks=$bl', 'kernel %.4f' % k, 'step %.4f' % d['ms_per_step'],
      'copy_floor %.4f' % cf.get('ms', 0), 'of_copy %.3f' % (cf.get('ms', 0) / k), flush=True)" || exit 1
  done
done
