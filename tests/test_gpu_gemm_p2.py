"""The two-workgroups-per-CU wide GEMM (csrc/gemm_p2.h, asrx_set_gemm_variant(1), the default) against the
one-workgroup-per-CU kernel (gemm_wr.h, variant 0): the same operand images, MFMA fragments, k order and
epilogue per wave, so every product is BIT-IDENTICAL -- for each epilogue it takes (bias, activation, saved
pre-activation, beta, bf16 C, residual add, MSheath row-tile lists) -- and both equal a float64 product of
the bf16-rounded operands within fp32 accumulation error (the projections of model.py:242-245, 421-425,
573-580)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _both(fn):
    """fn() under the p2 kernel and under the wr kernel -> (p2 result, wr result)."""
    from asrx import lib

    old = lib.load().asrx_set_gemm_variant(1)
    try:
        a = fn()
        lib.load().asrx_set_gemm_variant(0)
        b = fn()
    finally:
        lib.load().asrx_set_gemm_variant(old)
    return a, b


def _ref(x, W, b):
    xb = x.to(torch.bfloat16).double()
    return xb @ W.to(torch.bfloat16).double().t() + (b.double() if b is not None else 0.0)


@pytest.mark.parametrize("nj", [2, 3])
@pytest.mark.parametrize("abf", [False, True])
@pytest.mark.parametrize("M,N,K", [(5000, 384, 384), (257, 200, 96), (1000, 1152, 64), (8192, 1536, 384),
                                   (3001, 384, 1536), (130, 768, 384)])
@pytest.mark.parametrize("act", ["none", "gelu", "silu"])
def test_p2_matches_wr(cuda, nj, abf, M, N, K, act):
    from asrx import gemm as G

    g = torch.Generator().manual_seed(M + N + K + nj + 7 * abf)
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

    G._nj_override = nj
    try:
        (y1, z1), (y0, z0) = _both(run)
    finally:
        G._nj_override = None
    assert torch.equal(y1, y0) and torch.equal(z1, z0)
    ref = _ref(x, W, b)
    err = float((z1.double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err


@pytest.mark.parametrize("abf", [False, True])
def test_p2_beta_and_bf16_c(cuda, abf):
    from asrx import gemm as G

    M, N, K = 4099, 384, 384
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


def test_p2_residual_epilogue(cuda):
    """asrx_gemm_wn_res (the out projection's residual add, model.py:578-580) on both kernels."""
    from asrx import lib, ops

    M, N, K = 6001, 384, 384
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    r = torch.randn(M, N, generator=g).to(cuda)
    from asrx import gemm as G

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
    del ops


def test_p2_row_tiles(cuda):
    """MSheath's row-list launches (only the 128-row tiles of samples at a layer, model.py:441-482): rows of
    other tiles are left untouched by both kernels."""
    from asrx import gemm as G

    B, L, D = 7, 700, 384
    M = B * L
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, D, generator=g).to(cuda)
    W = (torch.randn(D, D, generator=g) / D ** 0.5).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    next_i = torch.tensor([0, 1, 1, 0, 2, 1, 0], dtype=torch.float32, device=cuda)
    tl, cnt = G.row_tiles(next_i, 1, L, M)

    def run():
        y = torch.full((M, D), 7.0, device=cuda)
        G.gemm_wn(x, Wb, y, M=M, N=D, K=D, lda=D, ldc=D, mtiles=(tl, cnt))
        return y

    G._nj_override = 3
    try:
        y1, y0 = _both(run)
    finally:
        G._nj_override = None
    assert torch.equal(y1, y0)
    ref = _ref(x, W, None).float()
    rows = torch.zeros(M, dtype=torch.bool, device=cuda)
    for t in tl[:int(cnt.item())].tolist():
        rows[t * 128:(t + 1) * 128] = True
    assert rows.any() and not rows.all()
    assert torch.allclose(y1[rows], ref[rows], rtol=1e-4, atol=1e-4)
    assert bool((y1[~rows] == 7.0).all())
