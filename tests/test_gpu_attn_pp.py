"""The software-pipelined flash-attention forward (attn_fwd_pp_kernel, asrx_set_attn_variant(1), the default
for multi-block launches at head dim 64) against the unpipelined kernel (variant 0): the same products in
the same order, so o and lse are BIT-IDENTICAL; and both against float64 SDPA of the bf16-rounded operands
(model.py:307 F.scaled_dot_product_attention, is_causal as the reference passes it)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(q, k, v, causal, variant, out_bf16):
    from asrx import lib, ops, prec

    old = lib.load().asrx_set_attn_variant(variant)
    try:
        with prec.precision("bf16"), torch.no_grad():
            o = ops.attention(q, k, v, causal, out_bf16=out_bf16)
    finally:
        lib.load().asrx_set_attn_variant(old)
    return o


@pytest.mark.parametrize("B,H,Lq,Lk,causal", [(2, 3, 3001, 3001, False), (3, 2, 700, 513, False),
                                              (2, 2, 777, 777, True), (1, 2, 257, 1000, False),
                                              (2, 6, 256, 64, False), (1, 1, 600, 65, True)])
@pytest.mark.parametrize("bf16_in", [False, True])
def test_attn_pp_bit_identical(cuda, B, H, Lq, Lk, causal, bf16_in):
    g = torch.Generator().manual_seed(B * 1000 + Lq + Lk)
    q, k, v = (torch.randn(B, L, H, 64, generator=g).to(cuda) for L in (Lq, Lk, Lk))
    q = q * 3.0  # scores well past 1: the lazy-rescale path runs
    if bf16_in:
        q, k, v = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
    o1 = _run(q, k, v, causal, 1, out_bf16=bf16_in)
    o0 = _run(q, k, v, causal, 0, out_bf16=bf16_in)
    assert torch.equal(o1, o0)
    qd, kd, vd = (t.to(torch.bfloat16).double().permute(0, 2, 1, 3).cpu() for t in (q, k, v))
    s = qd @ kd.transpose(-1, -2) / math.sqrt(64)
    if causal:
        s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool).triu(1), float("-inf"))
    ref = (torch.softmax(s, -1) @ vd).permute(0, 2, 1, 3)
    err = float((o1.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 3e-2, err
