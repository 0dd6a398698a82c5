#!/usr/bin/env python3
"""ISA check: for every kernel of the given HIP sources, count global loads that are
waited for (s_waitcnt vmcnt(0)) by the very next instruction — a load pattern the
compiler serialised (typically a conditional load `i < n ? p[i] : x` lowered to a branch
per element), so that each load is a full memory round trip."""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def check(src: Path):
    asm = Path("/tmp") / (src.stem + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-munsafe-fp-atomics", "-I", str(ROOT / "include"), "-S", "--cuda-device-only", str(src), "-o",
                    str(asm)], check=True, capture_output=True)
    s = asm.read_text()
    for name in re.findall(r"^(_Z\w+):", s, re.M):
        a = s.index(name + ":")
        b = s.find(".Lfunc_end", a)
        body = [l.strip() for l in s[a:b].splitlines()]
        loads = [i for i, l in enumerate(body) if l.startswith(("global_load", "buffer_load"))]
        ser = sum(1 for i in loads if i + 1 < len(body) and "vmcnt(0)" in body[i + 1])
        if loads:
            print(f"{src.name:18s} {name[:70]:70s} loads {len(loads):3d} serialised {ser:3d}")


if __name__ == "__main__":
    for f in sys.argv[1:] or sorted((ROOT / "nutdb_amd" / "csrc").glob("*.hip")):
        check(Path(f))
