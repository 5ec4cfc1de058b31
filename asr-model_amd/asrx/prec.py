"""Precision mode of the HIP path (SURVEY.md §8(b) "Precision modes").

"bf16"  (perf): GEMM / attention operands rounded to bf16, MFMA bf16 with fp32 accumulate; an
                activation whose only consumers are GEMM or attention operands (AbbyNormal outputs
                feeding a projection, per-head q / k, v, the attention output, GELU / SiLU outputs
                between two Linears, MSheath's LayerNorm outputs feeding its adapter / MLP) is
                stored bf16 by its producer -- the consumers rounded it to bf16 anyway, so the
                products are unchanged and the bytes halve; the residual stream, norm inputs and
                everything a backward reads for its own arithmetic stay fp32.
"fp32"  (parity): exact fp32 MFMA (v_mfma_f32_16x16x4_f32) everywhere.
"x3"    (reference-faithful training): storage and every kernel as "fp32", but the GEMMs run split-bf16 products
                (hi*hi + hi*lo + lo*hi of x = bf16 hi + bf16 lo, ~16-bit operands; csrc/gemm.hip PREC_X3) on the
                bf16 MFMA; attention stays exact fp32.  The float64 oracle with every GEMM / attention operand
                rounded to a hi + lo pair keeps the whole-gradient cosine at 0.993 where one bf16 rounding gives
                0.35 (profiles/r05_split_bf16_sensitivity.txt): the gradient mode that follows the reference's.

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
PREC_X3 = 3  # asrx_gemm only (split-bf16 products); everything else runs as PREC_F32
_NAMES = {"bf16": PREC_BF16, "fp32": PREC_F32, "x3": PREC_X3}

_mode = {"prec": PREC_BF16, "attn": "bf16", "store": True}


def set_precision(name: str) -> None:
    if name not in _NAMES:
        raise ValueError(f"precision must be 'bf16', 'fp32' or 'x3', got {name!r}")
    _mode["prec"] = _NAMES[name]


def get() -> int:
    return _mode["prec"]


def state() -> tuple:
    """Every switch of this module (a key for launch sequences recorded under one mode, e.g. the dead-block
    graphs of asrx.model.processor)."""
    return tuple(sorted(_mode.items()))


def name() -> str:
    return {v: k for k, v in _NAMES.items()}[_mode["prec"]]


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
    """Precision code for asrx_attn_fwd: fp8 only on top of the bf16 perf mode; x3 runs exact fp32 attention."""
    if _mode["attn"] == "fp8" and _mode["prec"] == PREC_BF16:
        return PREC_FP8ATT
    return attention_bwd_prec()


def attention_bwd_prec() -> int:
    """Precision code for asrx_attn_bwd (fp8 is forward only: its backward runs the bf16 kernels)."""
    return PREC_F32 if _mode["prec"] == PREC_X3 else _mode["prec"]


@contextlib.contextmanager
def attention(name_: str):
    old = _mode["attn"]
    set_attention(name_)
    try:
        yield
    finally:
        _mode["attn"] = old
