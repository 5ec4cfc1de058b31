"""Precision mode of the HIP path (SURVEY.md §8(b) "Precision modes").

"bf16"  (perf): GEMM / attention operands rounded to bf16 in LDS, MFMA bf16 with fp32 accumulate;
                activations, reductions and norms stay fp32 in HBM.
"fp32"  (parity): exact fp32 MFMA (v_mfma_f32_16x16x4_f32) everywhere.

Both modes run the same kernels (templated on the MFMA type); there is no CPU path.
"""
from __future__ import annotations

import contextlib

PREC_F32 = 0
PREC_BF16 = 1

_mode = {"prec": PREC_BF16}


def set_precision(name: str) -> None:
    if name not in ("bf16", "fp32"):
        raise ValueError(f"precision must be 'bf16' or 'fp32', got {name!r}")
    _mode["prec"] = PREC_BF16 if name == "bf16" else PREC_F32


def get() -> int:
    return _mode["prec"]


def name() -> str:
    return "bf16" if _mode["prec"] == PREC_BF16 else "fp32"


@contextlib.contextmanager
def precision(name_: str):
    old = _mode["prec"]
    set_precision(name_)
    try:
        yield
    finally:
        _mode["prec"] = old
