"""The nut_ctx option table is spelled in four places — the enum in include/nutexec.h, the
defaults in csrc/common.hpp, the accepted ranges in csrc/api.hip and Executor.OPTIONS —
and they must agree entry by entry (CPU only: source text and the Python table)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _enum():
    text = (ROOT / "include" / "nutexec.h").read_text()
    pairs = re.findall(r"NUT_OPT_([A-Z0-9_]+) = (\d+)", text)
    return {name.lower(): int(v) for name, v in pairs}


def _array(text, pattern):
    m = re.search(pattern + r"\s*=\s*\{([^}]*)\}", text)
    assert m, pattern
    return [int(x) for x in m.group(1).split(",")]


def test_enum_is_dense_and_counted():
    e = _enum()
    count = e.pop("count")
    assert sorted(e.values()) == list(range(count))


def test_executor_table_matches_enum():
    from nutdb_amd.executor import Executor
    e = _enum()
    e.pop("count")
    assert Executor.OPTIONS == e


def test_defaults_and_ranges_cover_every_option():
    e = _enum()
    count = e["count"]
    common = (ROOT / "nutdb_amd" / "csrc" / "common.hpp").read_text()
    api = (ROOT / "nutdb_amd" / "csrc" / "api.hip").read_text()
    defaults = _array(common, r"int64_t opt\[NUT_OPT_COUNT\]")
    lo = _array(api, r"lo\[NUT_OPT_COUNT\]")
    hi = _array(api, r"hi\[NUT_OPT_COUNT\]")
    assert len(defaults) == len(lo) == len(hi) == count
    for i, (d, a, b) in enumerate(zip(defaults, lo, hi)):
        assert a <= b, i
        # a default outside the settable range could never be restored by set_option
        assert a <= d <= b, (i, d, a, b)
