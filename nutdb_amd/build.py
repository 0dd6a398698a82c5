"""Build libnutexec.so (HIP kernels + C ABI) for gfx950, in-tree.

The shared library is the product: nutdb_amd/__init__.py loads it with ctypes and
fails loudly when it is missing.  Cross-compiles without a GPU.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libnutexec.so"
ARCH = "gfx950"

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",      # exact f64 arithmetic (parity with the CPU oracle)
    "-munsafe-fp-atomics",    # hardware ds_add_f64 / global_atomic_add_f64 (no CAS loops)
    "-Wall",
    "-Wno-unused-result",
]


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))


def build(force: bool = False, verbose: bool = False) -> Path:
    srcs = sources()
    deps = srcs + sorted(CSRC.glob("*.hpp")) + [ROOT / "include" / "nutexec.h"]
    if LIB.exists() and not force:
        mt = LIB.stat().st_mtime
        if all(p.stat().st_mtime <= mt for p in deps):
            return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *HIPCC_FLAGS, "-I", str(ROOT / "include"), *map(str, srcs), "-o", str(LIB) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(str(LIB) + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
