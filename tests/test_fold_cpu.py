"""The ordered group-by's host fold (nutdb_amd/csrc/fold.hpp: overflow-arena groups and
unplaced heavy keys merged into the key-sorted result) against a std::map merge, built
with g++ — serial and threaded block moves (tests/c/test_fold.cpp)."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_fold_sorted_groups(tmp_path):
    exe = tmp_path / "test_fold"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", str(ROOT / "nutdb_amd" / "csrc"),
                    str(ROOT / "tests" / "c" / "test_fold.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
