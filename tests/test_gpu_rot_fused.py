"""The q / k projections with rotary fused into the GEMM epilogue (asrx_gemm_wn_rot; model.py:242-245, 261 and
198-214 with the hd^-0.25 scale of model.py:303-304) against the projection GEMM followed by the separate
rotary pass (asrx_rotary_fwd2): the epilogue rotates the same fp32 product with the same unfused arithmetic,
so the outputs -- the rotated projection and the saved unrotated one -- are BIT-IDENTICAL, at the text side's
tile width (nj 1) and the audio side's (nj 3), bf16- and fp32-stored inputs; the autograd paths
(ops.linear_rotary, ops.kv_proj_rotary) give the unfused path's gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(cuda, B, L, D, abf, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, L, D, generator=g).to(cuda)
    src = torch.randn(B, L, D, generator=g).to(cuda)
    W = (torch.randn(D, D, generator=g) / D ** 0.5).to(cuda)
    b = torch.randn(D, generator=g).to(cuda)
    return (x.to(torch.bfloat16) if abf else x), src, W, b


@pytest.mark.parametrize("B,L", [(4, 256), (16, 3001), (3, 77)])  # nj 1, nj 3, ragged rows
@pytest.mark.parametrize("abf", [True, False])
@pytest.mark.parametrize("masked", [False, True])
def test_gemm_rot_matches_gemm_then_rotary(cuda, B, L, abf, masked):
    from asrx import gemm as G
    from asrx import lib, ops
    from asrx.model import rotary_freqs

    D, H = 384, 6
    hd = D // H
    x, src, W, b = _inputs(cuda, B, L, D, abf, B * L + abf + 2 * masked)
    freqs = rotary_freqs(D, H, masked, cuda)
    scale = hd ** -0.25
    m = torch.empty(B * L, device=cuda)
    lib.call("asrx_rownorm", lib.ptr(src), lib.ptr(m), B * L, D, lib.stream())
    tab = ops.rotary_table(freqs, L, hd)
    z = torch.empty(B, L, D, device=cuda)
    y = G.linear_rot_fwd(x, W, b, m, tab, L, hd, scale, preact=z)
    q = G.linear_fwd(x, W, b)
    ref = torch.empty_like(q)
    lib.call("asrx_rotary_fwd2", lib.ptr(q), lib.ptr(m), lib.ptr(freqs), lib.ptr(tab), lib.ptr(ref), B * L, L, D, hd,
             float(scale), lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(z, q)
    assert torch.equal(y, ref)
    y2 = G.linear_rot_fwd(x, W, b, m, tab, L, hd, scale)  # no saved product
    assert torch.equal(y2, ref)


def _grads(fused, fn, leaves):
    from asrx import ops

    old = ops.ROT_FUSED
    ops.ROT_FUSED = fused
    try:
        for t in leaves:
            t.grad = None
        out = fn()
        g = torch.Generator().manual_seed(5)
        w = [torch.randn(o.shape, generator=g).to(o.device) for o in out]
        sum((o.float() * wi).sum() for o, wi in zip(out, w)).backward()
        torch.cuda.synchronize()
        return [o.detach().float().clone() for o in out], [t.grad.clone() for t in leaves]
    finally:
        ops.ROT_FUSED = old


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("B,L", [(4, 256), (8, 3001)])
def test_linear_rotary_autograd_matches_unfused(cuda, B, L):
    from asrx import ops, prec
    from asrx.model import rotary_freqs

    D, H = 384, 6
    hd = D // H
    x0, src0, W, b = _inputs(cuda, B, L, D, False, 11 + L)
    W.requires_grad_(True)
    b.requires_grad_(True)
    x = x0.clone().requires_grad_(True)
    src = src0.clone().requires_grad_(True)
    freqs = rotary_freqs(D, H, True, cuda)
    with prec.precision("bf16"):
        def fn():
            return [ops.linear_rotary(x, W, b, src, freqs, hd, hd ** -0.25)]
        out_f, g_f = _grads(True, fn, [x, src, W, b])
        out_u, g_u = _grads(False, fn, [x, src, W, b])
    assert torch.equal(out_f[0], out_u[0])
    for gf, gu in zip(g_f, g_u):  # the same kernels in the same order; bias sums by atomics
        assert _rel(gf, gu) < 1e-5


@pytest.mark.parametrize("B,L", [(4, 256), (8, 3001)])
def test_kv_proj_rotary_autograd_matches_unfused(cuda, B, L):
    from asrx import ops, prec
    from asrx.model import rotary_freqs

    D, H = 384, 6
    hd = D // H
    g = torch.Generator().manual_seed(3 + L)
    x = torch.randn(B, L, D, generator=g).to(cuda).requires_grad_(True)
    src = torch.randn(B, L, D, generator=g).to(cuda).requires_grad_(True)
    W = (torch.randn(2 * D, D, generator=g) / D ** 0.5).to(cuda).requires_grad_(True)
    b = torch.randn(2 * D, generator=g).to(cuda).requires_grad_(True)
    freqs = rotary_freqs(D, H, False, cuda)
    with prec.precision("bf16"):
        def fn():
            k, v = ops.kv_proj_rotary(x, W, b, src, freqs, hd, hd ** -0.25)
            return [k, v]
        out_f, g_f = _grads(True, fn, [x, src, W, b])
        out_u, g_u = _grads(False, fn, [x, src, W, b])
    for a, c in zip(out_f, out_u):
        assert torch.equal(a, c)
    for gf, gu in zip(g_f, g_u):
        assert _rel(gf, gu) < 1e-5


@pytest.mark.parametrize("variant,B,L,abf", [(0, 16, 3001, True), (0, 16, 3001, False), (1, 48, 3001, False)])
def test_gemm_rot_every_wide_variant(cuda, variant, B, L, abf):
    """asrx_gemm_wn_rot under the A/B switch asrx_set_gemm_variant: variant 0 (gemm_wr only) and fp32 A at >= 131072
    rows (which gemm_p2 does not take) run the nj = 3 rotary epilogue on gemm_wr_kernel -- bit-identical to the
    GEMM + rotary pass like every other form (nj = 3 used to raise under variant 0)."""
    from asrx import gemm as G
    from asrx import lib, ops
    from asrx.model import rotary_freqs

    D, H = 384, 6
    hd = D // H
    x, src, W, b = _inputs(cuda, B, L, D, abf, 91 + variant + abf)
    freqs = rotary_freqs(D, H, False, cuda)
    scale = hd ** -0.25
    m = torch.empty(B * L, device=cuda)
    lib.call("asrx_rownorm", lib.ptr(src), lib.ptr(m), B * L, D, lib.stream())
    tab = ops.rotary_table(freqs, L, hd)
    old = lib.load().asrx_set_gemm_variant(variant)
    try:
        assert G._nj(B * L, D) == 3
        z = torch.empty(B, L, D, device=cuda)
        y = G.linear_rot_fwd(x, W, b, m, tab, L, hd, scale, preact=z)
        q = G.linear_fwd(x, W, b)
    finally:
        lib.load().asrx_set_gemm_variant(old)
    ref = torch.empty_like(q)
    lib.call("asrx_rotary_fwd2", lib.ptr(q), lib.ptr(m), lib.ptr(freqs), lib.ptr(tab), lib.ptr(ref), B * L, L, D, hd,
             float(scale), lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(z, q)
    assert torch.equal(y, ref)
