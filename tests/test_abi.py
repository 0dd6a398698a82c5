"""CPU checks of the drop-in boundary: libnutexec.so loads, exports every entry point
include/nutexec.h declares, and the ctypes struct layout equals the C layout.
No compute calls (no GPU here)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "nutexec.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nut_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    from nutdb_amd._lib import LIB_PATH, SIGNATURES
    lib = C.CDLL(str(LIB_PATH))
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), f"{name} declared in nutexec.h but not exported"
        assert name in SIGNATURES, f"{name} has no ctypes signature in nutdb_amd/_lib.py"


def test_no_torch_or_cxx_types_in_header():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)  # code only, not comments
    for bad in ("torch", "std::", "at::", "Tensor", "class ", "template"):
        assert bad not in text


def test_abi_version_and_error_string():
    from nutdb_amd._lib import lib
    assert lib.nut_abi_version() == 1
    # a call that fails argument validation before touching the GPU
    st = lib.nut_ctx_create(0, None)
    assert st == 1
    assert b"NULL" in lib.nut_last_error()


def test_struct_layout_matches_c(tmp_path):
    from nutdb_amd._lib import NutAggSpec
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "nutexec.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(nut_agg_spec),"
        " offsetof(nut_agg_spec,keys), offsetof(nut_agg_spec,pred_col), offsetof(nut_agg_spec,pred_i64),"
        " offsetof(nut_agg_spec,val_col), offsetof(nut_agg_spec,naggs), offsetof(nut_agg_spec,agg_expr),"
        " offsetof(nut_agg_spec,agg_arg));return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [C.sizeof(NutAggSpec), NutAggSpec.keys.offset, NutAggSpec.pred_col.offset, NutAggSpec.pred_i64.offset,
            NutAggSpec.val_col.offset, NutAggSpec.naggs.offset, NutAggSpec.agg_expr.offset,
            NutAggSpec.agg_arg.offset]
    assert got == want


def test_header_compiles_as_c_and_cxx(tmp_path):
    for comp, ext in (("gcc", "c"), ("g++", "cpp")):
        src = tmp_path / f"h.{ext}"
        src.write_text('#include "nutexec.h"\nint main(void){nut_ctx *c = 0; (void)c; return NUTEXEC_ABI_VERSION - 1;}\n')
        subprocess.run([comp, "-Wall", "-Werror", "-I", str(ROOT / "include"), "-c", str(src), "-o",
                        str(tmp_path / f"h_{ext}.o")], check=True)


def test_library_is_gfx950_code_object():
    from nutdb_amd._lib import LIB_PATH
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", str(LIB_PATH)], capture_output=True,
                         text=True).stdout
    assert ".hip_fatbin" in out
    blob = LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_dist_loads_rccl_and_fails_cleanly_without_gpu():
    """nut_dist_*: RCCL resolves (dlopen by soname) and makes a 128-byte unique id on a
    host without a GPU; creating ranks fails with a status, not a crash."""
    import torch
    from nutdb_amd import NutError
    from nutdb_amd.dist import NutDist
    assert len(NutDist.unique_id()) == 128
    if torch.cuda.is_available():
        return
    for make in (lambda: NutDist.virtual(2), lambda: NutDist.create([0])):
        try:
            make()
        except NutError as e:
            assert e.status != 0
        else:
            raise AssertionError("nut_dist created without a GPU")
