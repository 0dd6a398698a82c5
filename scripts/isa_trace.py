#!/usr/bin/env python3
"""Condensed memory-op trace of one kernel's gfx950 ISA: runs of global / scratch / LDS
ops, vmcnt waits and barriers, one line per run, so that a prefetch that waits for its
own data (a vmcnt wait right after the loads) or a spill inside the loop shows at a glance.
  scripts/isa_trace.py SRC.hip KERNEL_SUBSTRING [-D...]"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OPS = ("global_load", "global_store", "global_atomic", "scratch_load", "scratch_store", "ds_write", "ds_read",
       "ds_add", "buffer_load", "buffer_store", "s_waitcnt vmcnt", "s_barrier")


def main():
    src, pat, extra = Path(sys.argv[1]), sys.argv[2], sys.argv[3:]
    asm = Path("/tmp") / (src.stem + ".trace.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-munsafe-fp-atomics", "-I", str(ROOT / "include"), "-S", "--cuda-device-only", *extra, str(src),
                    "-o", str(asm)], check=True, capture_output=True)
    lines = asm.read_text().split("\n")
    starts = [(i, re.search(r"\.type\s+(\S+),@function", l).group(1)) for i, l in enumerate(lines) if "@function" in l]
    starts.append((len(lines), "END"))
    for (a, name), (b, _) in zip(starts, starts[1:]):
        if pat not in name:
            continue
        print("==", name)
        prev, cnt, at = None, 0, 0
        for i in range(a, b):
            l = lines[i].strip()
            key = next((p for p in OPS if l.startswith(p)), None)
            if l.startswith(".LBB") and "Loop Header" in l:
                key = "loop " + l.split(":")[0]
            if key and key == prev:
                cnt += 1
                continue
            if prev:
                print(f"{at - a:6d} {prev} x{cnt}")
            prev, cnt, at = key, 1, i
        if prev:
            print(f"{at - a:6d} {prev} x{cnt}")


if __name__ == "__main__":
    main()
