#!/usr/bin/env python3
"""Register / LDS / occupancy audit of every kernel in the given HIP sources (gfx950):
scripts/vgpr_audit.py SRC... — waves per SIMD = min(8, 512 // VGPRs rounded up to 8),
workgroups per CU from waves and LDS (160 KB).  A kernel that crosses a step (e.g. 128 ->
132 VGPRs: 4 -> 3 waves) halves its latency hiding without any other sign."""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def audit(src: Path):
    asm = Path("/tmp") / (src.stem + ".audit.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-munsafe-fp-atomics", "-I", str(ROOT / "include"), "-S", "--cuda-device-only", str(src), "-o",
                    str(asm)], check=True, capture_output=True)
    s = asm.read_text()
    meta = s[s.find("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - ", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or name.group(1).endswith(".kd"):
            continue
        g = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1)) if re.search(rf"\.{k}:\s+(\d+)", blk) else 0
        v, agpr, lds, wg = g("vgpr_count"), g("agpr_count"), g("group_segment_fixed_size"), g("max_flat_workgroup_size")
        scratch = g("private_segment_fixed_size")
        regs = -(-max(v, 1) // 8) * 8
        waves = min(8, 512 // regs)
        wpw = max(1, -(-wg // 64))
        per_cu = min(waves * 4 // wpw, (160 * 1024) // lds if lds else 99)
        print(f"{src.name:16s} vgpr {v:3d} agpr {agpr:3d} scratch {scratch:4d} lds {lds:6d} wg {wg:4d} "
              f"waves/SIMD {waves} wg/CU {per_cu:2d}  {name.group(1)[:80]}")


if __name__ == "__main__":
    for a in sys.argv[1:]:
        audit(Path(a))
