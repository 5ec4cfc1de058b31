"""Precision mode of the HIP path (SURVEY.md §8(b) "Precision modes").

"bf16"  (perf): GEMM / attention operands rounded to bf16, MFMA bf16 with fp32 accumulate; an
                activation whose only consumers are GEMM or attention operands (AbbyNormal outputs
                feeding a projection, per-head q / k, v, the attention output, GELU / SiLU outputs
                between two Linears, MSheath's LayerNorm outputs feeding its adapter / MLP) is
                stored bf16 by its producer -- the consumers rounded it to bf16 anyway, so the
                products are unchanged and the bytes halve; the residual stream, norm inputs and
                everything a backward reads for its own arithmetic stay fp32.
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

_mode = {"prec": PREC_BF16, "attn": "bf16", "store": True}


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


def bf16_storage() -> bool:
    """Producers write GEMM-only activations as bf16 (perf mode, unless switched off for A/B)."""
    return _mode["prec"] == PREC_BF16 and _mode["store"]


def attn_bf16_io() -> bool:
    """q / k / v / o in bf16: the bf16 flash kernels (the fp8 forward reads fp32 q / k)."""
    return bf16_storage() and _mode["attn"] == "bf16"


@contextlib.contextmanager
def storage(on: bool):
    """Switch bf16 activation storage on / off (A/B timing and the storage-equivalence tests)."""
    old = _mode["store"]
    _mode["store"] = bool(on)
    try:
        yield
    finally:
        _mode["store"] = old


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
