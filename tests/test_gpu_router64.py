"""The AbbyNormal router at d = 64 (csrc/gemm_wn.hip router64_kernel: logits = SiLU(x W1^T + b1) W2^T, the per-head
norms' mode_router of essentials.py:155-161) against the gemm_wr_kernel router epilogue it replaces
(asrx_set_gemm_variant(5 | 16)): the same fragments, k order, epilogue expressions and logit sum order, so h_pre
and the logits are BIT-IDENTICAL, for ragged row counts, with and without h_pre, with and without the bias; and
both equal a float64 product of the bf16-rounded operands within fp32 accumulation error."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).double()


@pytest.mark.parametrize("M", [1, 15, 16, 777, 49152, 200003])
@pytest.mark.parametrize("keep", [False, True])
@pytest.mark.parametrize("bias", [False, True])
def test_router64_bit_identical(cuda, M, keep, bias):
    from asrx import gemm as G
    from asrx import lib

    g = torch.Generator().manual_seed(M + 2 * keep + bias)
    x = torch.randn(M, 64, generator=g).to(cuda)
    W1 = (torch.randn(64, 64, generator=g) / 8).to(cuda)
    b1 = torch.randn(64, generator=g).to(cuda) if bias else torch.zeros(64, device=cuda)
    W2 = (torch.randn(3, 64, generator=g) / 8).to(cuda)
    old = lib.load().asrx_set_gemm_variant(5)
    try:
        h1, l1 = G.router_fwd(x, W1, b1, W2, keep)
        lib.load().asrx_set_gemm_variant(5 | 16)
        h0, l0 = G.router_fwd(x, W1, b1, W2, keep)
    finally:
        lib.load().asrx_set_gemm_variant(old)
    assert torch.equal(l1, l0)
    if keep:
        assert torch.equal(h1, h0)
    ref_h = _bf(x.cpu()) @ _bf(W1.cpu()).t() + b1.cpu().double()
    ref_l = torch.nn.functional.silu(ref_h) @ W2.cpu().double().t()
    assert float((l1.cpu().double() - ref_l).abs().max() / ref_l.abs().max()) < 1e-5
