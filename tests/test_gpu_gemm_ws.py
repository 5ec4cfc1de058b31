"""The weight-stationary wide GEMM (csrc/gemm_ws.h; in the default variant 5 for launches with K <= 384, K % 64
== 0, >= 32768 rows and bf16 A at N >= 768 or fp32 A at N <= 768; variant 13 = every shape it can run, what these
tests use) against the two-workgroups-per-CU kernel (variant 1): the same MFMA fragments and
k order per output element and the same epilogue code, so every product is BIT-IDENTICAL -- for each epilogue
it takes (bias, activation, saved pre-activation, alpha / beta, bf16 C, residual add, rotary) and for partial
column slices and ragged row tiles -- and both equal a float64 product of the bf16-rounded operands within fp32
accumulation error (the projections of model.py:242-245, 421-425, 573-580)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _both(fn):
    """fn() under the weight-stationary kernel and under gemm_p2 -> (ws result, p2 result)."""
    from asrx import lib

    old = lib.load().asrx_set_gemm_variant(13)
    try:
        a = fn()
        lib.load().asrx_set_gemm_variant(1)
        b = fn()
    finally:
        lib.load().asrx_set_gemm_variant(old)
    return a, b


def _ref(x, W, b):
    xb = x.to(torch.bfloat16).double()
    return xb @ W.to(torch.bfloat16).double().t() + (b.double() if b is not None else 0.0)


@pytest.mark.parametrize("abf", [False, True])
@pytest.mark.parametrize("M,N,K", [(32768, 384, 384), (48017, 384, 384), (40000, 200, 256), (33000, 1536, 384),
                                   (36001, 1152, 64), (32800, 256, 384), (40000, 768, 384), (34000, 776, 128)])
@pytest.mark.parametrize("act", ["none", "gelu", "silu", "sigmoid"])
def test_ws_matches_p2(cuda, abf, M, N, K, act):
    from asrx import gemm as G

    g = torch.Generator().manual_seed(M + N + K + 7 * abf)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    xa = x.to(torch.bfloat16) if abf else x

    def run():
        y = torch.empty(M, N, device=cuda)
        z = torch.empty(M, N, device=cuda)
        G.gemm_wn(xa, Wb, y, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act=act, Z=z)
        return y, z

    (y1, z1), (y0, z0) = _both(run)
    assert torch.equal(z1, z0) and torch.equal(y1, y0)
    ref = _ref(x, W, b)
    err = float((z1.double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err


@pytest.mark.parametrize("abf", [False, True])
def test_ws_beta_and_bf16_c(cuda, abf):
    from asrx import gemm as G

    M, N, K = 40999, 384, 384
    g = torch.Generator().manual_seed(11)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    c0 = torch.randn(M, N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    xa = x.to(torch.bfloat16) if abf else x

    def run():
        y = c0.clone()
        G.gemm_wn(xa, Wb, y, M=M, N=N, K=K, lda=K, ldc=N, alpha=0.5, beta=1.0)
        yb = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        G.gemm_wn(xa, Wb, yb, M=M, N=N, K=K, lda=K, ldc=N, act="silu")
        return y, yb

    (y1, b1), (y0, b0) = _both(run)
    assert torch.equal(y1, y0) and torch.equal(b1, b0)
    ref = 0.5 * _ref(x, W, None) + c0.double()
    assert float((y1.double() - ref).abs().max() / ref.abs().max()) < 1e-5


def test_ws_residual_epilogue(cuda):
    """asrx_gemm_wn_res (the out projection's residual add, model.py:578-580) on both kernels."""
    from asrx import gemm as G
    from asrx import lib

    M, N, K = 60001, 384, 384
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    r = torch.randn(M, N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)

    def run():
        y = torch.empty(M, N, device=cuda)
        lib.call("asrx_gemm_wn_res", lib.ptr(x), K, lib.ptr(Wb), Wb.stride(0), lib.ptr(y), N, lib.ptr(b), lib.ptr(r),
                 N, M, N, K, 3, lib.stream())
        return y

    y1, y0 = _both(run)
    assert torch.equal(y1, y0)
    ref = _ref(x, W, b) + r.double()
    assert float((y1.double() - ref).abs().max() / ref.abs().max()) < 1e-5


@pytest.mark.parametrize("abf", [False, True])
def test_ws_rotary_epilogue(cuda, abf):
    """asrx_gemm_wn_rot (q / k projection + rotary, model.py:198-214) on both kernels, with the saved product."""
    from asrx import gemm as G
    from asrx import lib, ops
    from asrx.model import rotary_freqs

    B, L, D, H = 12, 3001, 384, 6
    hd = D // H
    g = torch.Generator().manual_seed(9 + abf)
    x = torch.randn(B, L, D, generator=g).to(cuda)
    src = torch.randn(B, L, D, generator=g).to(cuda)
    W = (torch.randn(D, D, generator=g) / D ** 0.5).to(cuda)
    b = torch.randn(D, generator=g).to(cuda)
    xa = x.to(torch.bfloat16) if abf else x
    freqs = rotary_freqs(D, H, False, cuda)
    m = torch.empty(B * L, device=cuda)
    lib.call("asrx_rownorm", lib.ptr(src), lib.ptr(m), B * L, D, lib.stream())
    tab = ops.rotary_table(freqs, L, hd)

    def run():
        z = torch.empty(B, L, D, device=cuda)
        y = G.linear_rot_fwd(xa, W, b, m, tab, L, hd, hd ** -0.25, preact=z)
        return y, z

    (y1, z1), (y0, z0) = _both(run)
    assert torch.equal(z1, z0) and torch.equal(y1, y0)
