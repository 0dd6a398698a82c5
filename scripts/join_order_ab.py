"""Ordered vs unordered probe of the bench's join workload (1e9 probe x 2.5e8 build keys):
wall time per join (torch events around the whole call) and the pair count of each mode.
usage: python scripts/join_order_ab.py [rows] [reps]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import Join  # noqa: E402
from nutdb_amd.executor import Executor  # noqa: E402


def main():
    rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**9
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ex = Executor(0)
    j = Join(ex, rows, 0)
    torch.cuda.synchronize()
    for any_order in (False, True, False, True):
        ts = []
        for r in range(reps + 1):
            t0 = time.perf_counter()
            pi, bi = ex.join_i64(j.build, j.probe, "inner", any_order=any_order)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            n = pi.numel()
            del pi, bi
        ts = sorted(ts[1:])
        print(f"any_order={int(any_order)} pairs={n} ms min {ts[0]:.2f} median {ts[len(ts) // 2]:.2f}", flush=True)


if __name__ == "__main__":
    main()
