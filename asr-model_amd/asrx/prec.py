"""Precision mode of the HIP path (SURVEY.md §8(b) "Precision modes").

"bf16"  (perf): GEMM / attention operands rounded to bf16 in LDS, MFMA bf16 with fp32 accumulate;
                activations, reductions and norms stay fp32 in HBM.
"fp32"  (parity): exact fp32 MFMA (v_mfma_f32_16x16x4_f32) everywhere.

Attention mode (orthogonal, perf mode only): "fp8" runs the attention forward with QK^T on OCP e4m3
(per-row scales, MX-rate MFMA; softmax and PV stay bf16) -- SURVEY.md §8(b) config 5 (fp8 attention,
greedy decode).  Forward only: a backward through an fp8 forward runs the bf16 kernels.

Both modes run the same kernels (templated on the MFMA type); there is no CPU path.
"""
from __future__ import annotations

import contextlib

PREC_F32 = 0
PREC_BF16 = 1
PREC_FP8ATT = 2  # asrx_attn_fwd only

_mode = {"prec": PREC_BF16, "attn": "bf16"}


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


def set_attention(name_: str) -> None:
    if name_ not in ("bf16", "fp8"):
        raise ValueError(f"attention mode must be 'bf16' or 'fp8', got {name_!r}")
    _mode["attn"] = name_


def attention_prec() -> int:
    """Precision code for asrx_attn_fwd: fp8 only on top of the bf16 perf mode."""
    if _mode["attn"] == "fp8" and _mode["prec"] == PREC_BF16:
        return PREC_FP8ATT
    return _mode["prec"]


@contextlib.contextmanager
def attention(name_: str):
    old = _mode["attn"]
    set_attention(name_)
    try:
        yield
    finally:
        _mode["attn"] = old
