"""The software-pipelined attention forward (csrc/attn_mf.hip attn_fwd_sp_kernel, asrx_set_attn_variant(1), the
default at head dim 64) against the round-4 forward (variant 0): the same per-element arithmetic in the same
order, so the outputs, the log-sum-exp rows the backward reads, and therefore every gradient are BIT-IDENTICAL
-- for causal and non-causal masks, Lq != Lk, one partial tile, an odd and an even tile count (the loop is
unrolled by two), and fp32 or bf16 operands (F.scaled_dot_product_attention at model.py:307)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(q, k, v, causal, out_bf16):
    from asrx import ops, prec

    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    with prec.precision("bf16"):
        y = ops.attention(qr, kr, vr, causal, out_bf16=out_bf16)
        g = torch.autograd.grad(y, (qr, kr, vr), torch.ones_like(y) * 0.01 + y.detach() * 0.1)
    return (y.detach().float(),) + tuple(t.float() for t in g)


@pytest.mark.parametrize("B,H,Lq,Lk,causal", [(2, 3, 3001, 3001, False), (2, 2, 700, 1500, False),
                                              (1, 2, 1500, 700, True), (3, 2, 63, 63, False), (1, 1, 64, 64, False),
                                              (1, 2, 129, 129, True), (2, 2, 256, 2, False), (1, 2, 300, 192, False)])
@pytest.mark.parametrize("bf", [False, True])
def test_sp_forward_bit_identical(cuda, B, H, Lq, Lk, causal, bf):
    from asrx import lib

    g = torch.Generator().manual_seed(B * 1000 + Lq + Lk + causal)
    q = torch.randn(B, Lq, H, 64, generator=g).to(cuda)
    k = torch.randn(B, Lk, H, 64, generator=g).to(cuda)
    v = torch.randn(B, Lk, H, 64, generator=g).to(cuda)
    q[:, :, :, :8] *= 6.0  # spread the score scale so the lazy rescale fires on later tiles too
    if bf:
        q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    old = lib.load().asrx_set_attn_variant(1)
    try:
        a = _run(q, k, v, causal, bf)
        lib.load().asrx_set_attn_variant(0)
        b = _run(q, k, v, causal, bf)
    finally:
        lib.load().asrx_set_attn_variant(old)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    qb, kb, vb = (t.to(torch.bfloat16).float().transpose(1, 2) for t in (q, k, v))
    ref = torch.nn.functional.scaled_dot_product_attention(qb, kb, vb, is_causal=causal).transpose(1, 2)
    # P rounded to bf16 before the PV product (the kernel's documented precision): ~2^-9 relative per term
    err = float((a[0] - ref).abs().max() / ref.abs().max())
    assert err < 2e-2, err
