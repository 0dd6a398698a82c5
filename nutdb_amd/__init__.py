"""nutdb_amd — MI355X-native columnar executor for NutDB (hot path: scan/filter,
hash group-by aggregation, radix sort; multi-GPU group-by over RCCL).

Importing this package loads libnutexec.so (hand-written HIP for gfx950 behind the C
ABI in include/nutexec.h) and raises if it is missing: there is no CPU fallback.
"""
from ._lib import NutError, lib  # noqa: F401  (loads the HIP library or raises)
from .executor import Agg, AggQuery, Executor, Groups, ProgQuery  # noqa: F401

__all__ = ["Agg", "AggQuery", "Executor", "Groups", "NutError", "ProgQuery", "lib"]
