"""Build the C host programs under tests/c (test infrastructure): plain gcc against the
HIP runtime's C API, libnutexec.so and the oracle — no hipcc, no Python, no torch in the
resulting processes.  Binaries go to tests/c/bin/ (git-ignored; they travel to the GPU
box with the tree like the built libraries)."""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
BIN = HERE / "bin"


def build(force: bool = False) -> list[Path]:
    BIN.mkdir(exist_ok=True)
    lib_dirs = [ROOT / "nutdb_amd", ROOT / "oracle", Path("/opt/rocm/lib")]
    deps = [ROOT / "include" / "nutexec.h", ROOT / "oracle" / "oracle.h", ROOT / "nutdb_amd" / "libnutexec.so",
            ROOT / "oracle" / "liboracle.so"]
    out = []
    for src in sorted(HERE.glob("*.c")):
        exe = BIN / src.stem
        out.append(exe)
        if not force and exe.exists() and all(exe.stat().st_mtime >= p.stat().st_mtime for p in [src] + deps):
            continue
        cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I", str(ROOT / "include"),
               "-I", str(ROOT / "oracle"), "-I", "/opt/rocm/include", str(src), "-o", str(exe) + ".tmp"]
        for d in lib_dirs:
            cmd += ["-L", str(d), f"-Wl,-rpath,{d}"]
        cmd += ["-lnutexec", "-loracle", "-lamdhip64", "-lm"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"gcc {src.name} failed:\n{r.stdout}\n{r.stderr}")
        Path(str(exe) + ".tmp").replace(exe)
    return out


if __name__ == "__main__":
    for p in build(force=True):
        print(p)
