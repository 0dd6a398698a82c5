"""Shared test helpers: the golden script's numpy restatement + comparison utilities."""
import importlib.util
from pathlib import Path

import numpy as np

_spec = importlib.util.spec_from_file_location("make_golden", Path(__file__).parent / "golden" / "make_golden.py")
mg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mg)

gen = mg.gen
pos_hash = mg.pos_hash
multiset_hash = mg.multiset_hash
wsum = mg.wsum
OPS = mg.OPS
OPCODE = {"<": 0, "<=": 1, ">": 2, ">=": 3, "==": 4, "!=": 5}


def fromhex(xs):
    return np.array([float.fromhex(x) for x in xs], dtype=np.float64)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.maximum(np.abs(b), 1e-300)
    return np.max(np.abs(a - b) / den) if len(a) else 0.0


F64_SUM_RTOL = 1e-12  # BASELINE.json north_star: f64 sums within 1e-12 relative
