"""GPU parity of the GEMM and log-mel kernels (through the C-ABI)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(A, B):
    return (A.double() @ B.double()).float()


@pytest.mark.parametrize("prec,tol", [(0, 2e-5), (1, 2e-2)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_layouts(cuda, prec, tol, a_kc, b_kc):
    from asrx.gemm import gemm

    g = torch.Generator().manual_seed(0)
    M, N, K = 200, 136, 264
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    bias = torch.randn(N, generator=g)
    Ad = (A if a_kc else A.t().contiguous()).to(cuda)
    Bd = (B.t().contiguous() if b_kc else B).to(cuda)
    C = torch.empty(M, N, device=cuda)
    gemm(Ad, Bd, C, M=M, N=N, K=K, lda=K if a_kc else M, ldb=K if b_kc else N, ldc=N, a_kc=a_kc,
         b_kc=b_kc, bias=bias.to(cuda), precision=prec)
    ref = _ref(A, B) + bias
    err = (C.cpu() - ref).abs().max() / ref.abs().max()
    assert err < tol, err


@pytest.mark.parametrize("act", ["gelu", "silu", "sigmoid"])
def test_gemm_epilogue(cuda, act):
    from asrx.gemm import gemm

    g = torch.Generator().manual_seed(1)
    M, N, K = 64, 96, 32
    A, B = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    C = torch.empty(M, N, device=cuda)
    Z = torch.empty(M, N, device=cuda)
    gemm(A.to(cuda), B.to(cuda), C, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, act=act, Z=Z, precision=0)
    z = A.double() @ B.double().t()
    f = {"gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu, "sigmoid": torch.sigmoid}[act]
    assert torch.allclose(Z.cpu().double(), z, atol=1e-4)
    assert torch.allclose(C.cpu().double(), f(z), atol=1e-4)


def test_gemm_splitk_batched_beta(cuda):
    from asrx.gemm import gemm

    g = torch.Generator().manual_seed(2)
    Bt, M, N, K = 3, 64, 72, 1000
    A, B = torch.randn(Bt, M, K, generator=g), torch.randn(Bt, N, K, generator=g)
    C0 = torch.randn(Bt, M, N, generator=g)
    C = C0.clone().to(cuda)
    gemm(A.to(cuda), B.to(cuda), C, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, batch=Bt, sA=M * K, sB=N * K,
         sC=M * N, beta=1.0, splitk=4, precision=0)
    ref = C0.double() + A.double() @ B.double().transpose(1, 2)
    assert torch.allclose(C.cpu().double(), ref, rtol=1e-4, atol=1e-3)


def test_conv3_implicit_im2col(cuda):
    """k3/pad1 Conv1d on channels-last sequences == F.conv1d; dgrad + wgrad via the same kernel."""
    from asrx.gemm import gemm

    g = torch.Generator().manual_seed(3)
    Bn, T, Ci, Co = 2, 37, 8, 12
    x = torch.randn(Bn, Ci, T, generator=g, dtype=torch.float64)
    W = torch.randn(Co, Ci, 3, generator=g, dtype=torch.float64)
    ref = torch.nn.functional.conv1d(x, W, padding=1)  # (B, Co, T)
    xcl = x.transpose(1, 2).contiguous().float().to(cuda)  # (B, T, Ci)
    Wt = W.permute(0, 2, 1).reshape(Co, 3 * Ci).contiguous().float().to(cuda)  # [o][k*Ci + c]
    y = torch.empty(Bn * T, Co, device=cuda)
    gemm(xcl, Wt, y, M=Bn * T, N=Co, K=3 * Ci, lda=Ci, ldb=3 * Ci, ldc=Co, conv_a=True, conv_F=T,
         conv_C=Ci, precision=0)
    assert torch.allclose(y.cpu().double().view(Bn, T, Co).transpose(1, 2), ref, atol=1e-4)
    # wgrad: dW[o, k*Ci + c] = sum_t dy[t, o] x[t + k - 1, c]
    dy = torch.randn(Bn, Co, T, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    Wr = W.clone().requires_grad_(True)
    torch.nn.functional.conv1d(xr, Wr, padding=1).backward(dy)
    dycl = dy.transpose(1, 2).contiguous().float().to(cuda)
    dW = torch.zeros(Co, 3 * Ci, device=cuda)
    gemm(dycl, xcl, dW, M=Co, N=3 * Ci, K=Bn * T, lda=Co, ldb=Ci, ldc=3 * Ci, a_kc=False, b_kc=False,
         conv_b=True, conv_F=T, conv_C=Ci, beta=1.0, splitk=2, precision=0)
    assert torch.allclose(dW.cpu().double().view(Co, 3, Ci).permute(0, 2, 1), Wr.grad, atol=1e-3)
    # dgrad: dx = conv3(dy, W~), W~[c][k'*Co + o] = W[o][c][2-k']
    Wf = W.flip(2).permute(1, 2, 0).reshape(Ci, 3 * Co).contiguous().float().to(cuda)
    dx = torch.empty(Bn * T, Ci, device=cuda)
    gemm(dycl, Wf, dx, M=Bn * T, N=Ci, K=3 * Co, lda=Co, ldb=3 * Co, ldc=Ci, conv_a=True, conv_F=T,
         conv_C=Co, precision=0)
    assert torch.allclose(dx.cpu().double().view(Bn, T, Ci).transpose(1, 2), xr.grad, atol=1e-3)


def test_linear_helpers(cuda):
    from asrx import gemm as G

    g = torch.Generator().manual_seed(4)
    x = torch.randn(5, 33, 64, generator=g)
    W = torch.randn(48, 64, generator=g)
    b = torch.randn(48, generator=g)
    dy = torch.randn(5, 33, 48, generator=g)
    with __import__("asrx.prec", fromlist=["x"]).precision("fp32"):
        y = G.linear_fwd(x.to(cuda), W.to(cuda), b.to(cuda))
        dx = G.linear_dgrad(dy.to(cuda), W.to(cuda))
        dW = G.linear_wgrad(dy.to(cuda), x.to(cuda))
    assert torch.allclose(y.cpu(), x @ W.t() + b, atol=1e-4)
    assert torch.allclose(dx.cpu(), dy @ W, atol=1e-4)
    assert torch.allclose(dW.cpu(), dy.reshape(-1, 48).t() @ x.reshape(-1, 64), atol=1e-3)


def _clip(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    f = rng.uniform(100, 300)
    x = 0.5 * np.sin(2 * np.pi * f * t) * (1 + 0.3 * np.sin(2 * np.pi * 3 * t)) + 0.05 * rng.standard_normal(n)
    return (x / np.abs(x).max()).astype(np.float32)


@pytest.mark.parametrize("n", [16000, 480000, 12345])
def test_logmel_matches_oracle(cuda, n):
    from asrx.mel import logmel
    from oracle import mel as omel

    clips = np.stack([_clip(n, s) for s in range(3)])
    out_bfm = logmel(torch.from_numpy(clips).to(cuda), layout="BFM").cpu().numpy()
    out_bmf = logmel(torch.from_numpy(clips).to(cuda), layout="BMF").cpu().numpy()
    for b in range(3):
        ref = omel.log_mel(clips[b].astype(np.float64))
        assert out_bmf[b].shape == ref.shape
        assert np.array_equal(out_bmf[b], out_bfm[b].T)
        err = np.abs(out_bmf[b] - ref).max()
        assert err < 2e-4, err


def test_logmel_floor_on_some_tiles(cuda):
    """The clip-max floor (essentials.py:485-488) is applied by a second pass only to the 16-frame tiles
    that hold a value below max - 8 (asrx_logmel's logmel_floor_kernel): clips whose floor covers some
    tiles and not others -- loud noise followed by near-silence, and a pure tone whose far bands fall
    below the floor -- match the oracle, and the floored entries are exactly (max - 8 + 4) / 4."""
    from asrx.mel import logmel
    from oracle import mel as omel

    n = 48000
    t = np.arange(n) / 16000.0
    rng = np.random.default_rng(3)
    loud_then_quiet = np.where(t < 1.3, 0.5, 1e-6) * rng.standard_normal(n)  # broadband: no band floored while loud
    pure = 0.9 * np.sin(2 * np.pi * 440 * t)
    clips = np.stack([loud_then_quiet, pure, _clip(n, 11)]).astype(np.float32)
    out_bfm = logmel(torch.from_numpy(clips).to(cuda), layout="BFM").cpu().numpy()
    out_bmf = logmel(torch.from_numpy(clips).to(cuda), layout="BMF").cpu().numpy()
    floored_tiles = []
    for b in range(3):
        ref = omel.log_mel(clips[b].astype(np.float64))
        assert np.array_equal(out_bmf[b], out_bfm[b].T)
        assert np.abs(out_bmf[b] - ref).max() < 2e-4
        low = ref == ref.min()  # the floored entries (the floor is the clip's minimum)
        fmin = out_bmf[b][low]
        assert np.all(fmin == fmin[0]), "floored entries must share one value"
        # frames (16 per tile) that hold a floored entry
        tiles = np.unique(np.nonzero(low.any(axis=0))[0] // 16)
        floored_tiles.append((len(tiles), (ref.shape[1] + 15) // 16))
    # the quiet tail floors some tiles and leaves the loud ones alone
    assert 0 < floored_tiles[0][0] < floored_tiles[0][1], floored_tiles


def test_logmel_pool_and_silence(cuda):
    from asrx.mel import logmel
    from oracle import mel as omel

    clips = np.stack([_clip(480000, 7), np.zeros(480000, np.float32)])
    out, pooled = logmel(torch.from_numpy(clips).to(cuda), layout="BMF", pool=True)
    out, pooled = out.cpu().numpy(), pooled.cpu().numpy()
    assert np.all(out[1] == -1.5)
    ref = omel.waveform_feature(clips[0].astype(np.float64))[0]
    assert np.abs(pooled[0] - ref).max() < 1e-6
    assert np.all(pooled[1] == 0)


@pytest.mark.parametrize("M,N,K", [(1000, 384, 384), (300, 1152, 384), (4200, 384, 1536), (129, 64, 384),
                                   (777, 200, 96)])
def test_wide_gemm_bf16(cuda, M, N, K):
    """asrx_gemm_wn (bf16 weights, fp32 activations) for fwd, dgrad and the k3 conv path."""
    from asrx import gemm as G
    from asrx import prec

    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    with prec.precision("bf16"):
        G.clear_weight_cache()
        y = G.linear_fwd(x.to(cuda), W.to(cuda), b.to(cuda), act="gelu").cpu()
        dx = G.linear_dgrad(dy.to(cuda), W.to(cuda)).cpu()
    ref_y = torch.nn.functional.gelu(x.double() @ W.double().t() + b.double())
    ref_dx = dy.double() @ W.double()
    assert float((y.double() - ref_y).abs().max() / ref_y.abs().max()) < 2e-2
    assert float((dx.double() - ref_dx).abs().max() / ref_dx.abs().max()) < 2e-2


def test_wide_conv3_bf16(cuda):
    from asrx import ops, prec

    g = torch.Generator().manual_seed(5)
    Bn, T, C, O = 3, 101, 64, 136
    x = torch.randn(Bn, C, T, generator=g)
    W = torch.randn(O, C, 3, generator=g) / (3 * C) ** 0.5
    bias = torch.randn(O, generator=g)
    with prec.precision("bf16"):
        y = ops.Conv3.apply(x.transpose(1, 2).contiguous().to(cuda), None, W.to(cuda), bias.to(cuda)).cpu()
    ref = torch.nn.functional.conv1d(x.double(), W.double(), bias.double(), padding=1).transpose(1, 2)
    assert float((y.double() - ref).abs().max() / ref.abs().max()) < 2e-2


def _bf(t):
    return t.to(torch.bfloat16).double()


@pytest.mark.parametrize("nj", [1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(5000, 384, 384), (1000, 1152, 64), (257, 200, 96), (70000, 64, 384)])
def test_wide_gemm_exact_bf16_inputs(cuda, nj, M, N, K):
    """Persistent wide GEMM against float64 on the same bf16-rounded operands: only the fp32
    accumulation order differs, so the tolerance is tight.  Covers every tile width, partial tiles
    in M and N, bias + GELU with the pre-activation Z, and the beta (accumulate) epilogue."""
    from asrx import gemm as G
    from asrx import lib

    g = torch.Generator().manual_seed(M * 7 + N + K + nj)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    xg, Wg, bg = x.to(cuda), W.to(cuda), b.to(cuda)
    Wb = G.weight_bf16(Wg, cache=False)
    y = torch.empty(M, N, device=cuda)
    z = torch.empty(M, N, device=cuda)
    G._nj_override = nj
    try:
        G.gemm_wn(xg, Wb, y, M=M, N=N, K=K, lda=K, ldc=N, bias=bg, act="gelu", Z=z)
        acc = c0.to(cuda)
        G.gemm_wn(xg, Wb, acc, M=M, N=N, K=K, lda=K, ldc=N, alpha=0.5, beta=2.0)
    finally:
        G._nj_override = None
    ref_z = _bf(x) @ _bf(W).t() + b.double()
    ref_y = torch.nn.functional.gelu(ref_z)
    ref_acc = 0.5 * (_bf(x) @ _bf(W).t()) + 2.0 * c0.double()
    for got, ref in ((z, ref_z), (y, ref_y), (acc, ref_acc)):
        assert float((got.cpu().double() - ref).abs().max() / ref.abs().max()) < 2e-6


@pytest.mark.parametrize("M,N,keep", [(3001, 384, True), (12000, 384, False), (777, 64, True), (129, 256, False)])
def test_router_gemm(cuda, M, N, keep):
    """asrx_gemm_wn_router: h_pre = x W1^T + b1 and logits = SiLU(h_pre) W2^T fused in the GEMM
    epilogue (AbbyNormal mode_router, essentials.py:155-161), on bf16-rounded operands."""
    from asrx import gemm as G

    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, N, generator=g)
    W1 = torch.randn(N, N, generator=g) / N ** 0.5
    b1 = torch.randn(N, generator=g)
    W2 = torch.randn(3, N, generator=g) / N ** 0.5
    hpre, logits = G.router_fwd(x.to(cuda), W1.to(cuda), b1.to(cuda), W2.to(cuda), keep)
    ref_h = _bf(x) @ _bf(W1).t() + b1.double()
    ref_l = torch.nn.functional.silu(ref_h) @ W2.double().t()
    assert float((logits.cpu().double() - ref_l).abs().max() / ref_l.abs().max()) < 1e-5
    if keep:
        assert float((hpre.cpu().double() - ref_h).abs().max() / ref_h.abs().max()) < 2e-6
    else:
        assert hpre is None


def test_abby_fused_router_matches_unfused(cuda):
    """Perf-mode AbbyNormal: the fused router path (logits from the GEMM epilogue) selects the same
    normalisation per row as the two-kernel path and gives the same output."""
    from asrx import gemm as G
    from asrx import lib, ops, prec

    g = torch.Generator().manual_seed(3)
    rows, d = 6000, 384
    x = torch.randn(rows, d, generator=g).to(cuda) * 3
    W1 = (torch.randn(d, d, generator=g) / d ** 0.5).to(cuda)
    b1 = torch.randn(d, generator=g).to(cuda)
    W2 = (torch.randn(3, d, generator=g) / d ** 0.5).to(cuda)
    b2 = torch.randn(3, generator=g).to(cuda)
    with prec.precision("bf16"):
        fused = ops.AbbyNormalFn.apply(x, W1, b1, W2, b2, 3000, 1, 0, 1234, True, False)
        hpre = G.linear_fwd(x, W1, b1)
    out = torch.empty_like(x)
    ys = torch.empty(rows, 3, device=cuda)
    idx = torch.empty(rows, dtype=torch.int32, device=cuda)
    lib.call("asrx_abby_fwd", lib.ptr(x), lib.ptr(hpre), lib.ptr(W2), lib.ptr(b2), lib.ptr(out), lib.ptr(ys),
             lib.ptr(idx), rows, d, 3000, 1, 0, 1234, 1, lib.stream())
    same = (fused - out).abs().max(dim=1).values <= 1e-5 * out.abs().max()
    assert float(same.float().mean()) > 0.999  # only near-tie gumbel picks may differ


@pytest.mark.parametrize("L,N", [(300, 256), (129, 384), (1000, 64)])
def test_wide_gemm_row_tiles(cuda, L, N):
    """asrx_row_tiles + asrx_gemm_wn_rows (MSheath layers skip samples not at the layer): the tiles
    holding rows of active samples equal the full GEMM, every other row is left untouched."""
    from asrx import gemm as G, prec

    g = torch.Generator().manual_seed(11)
    B, K = 7, 384
    M = B * L
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    next_i = torch.tensor([2.0, 1.0, 2.0, 3.0, 3.0, 2.0, 0.0], device=cuda)
    layer = 2
    with prec.precision("bf16"):
        full = G.linear_fwd(x, W, bias)
        mt = G.row_tiles(next_i, layer, L, M)
        y = torch.full((M, N), 12345.0, device=cuda)
        G.linear_fwd(x, W, bias, out=y, mtiles=mt)
    tl, cnt = mt[0].cpu(), int(mt[1])
    want = [t for t in range((M + 127) // 128)
            if any(float(next_i[b]) == layer for b in range(t * 128 // L, (min(t * 128 + 128, M) - 1) // L + 1))]
    assert tl[:cnt].tolist() == want
    rows = torch.zeros(M, dtype=torch.bool)
    for t in want:
        rows[t * 128:min(t * 128 + 128, M)] = True
    rows = rows.to(cuda)
    assert torch.equal(y[rows], full[rows])
    assert bool((y[~rows] == 12345.0).all())


@pytest.mark.parametrize("R,M,N,ld_extra", [(8192, 384, 384, 0), (777, 64, 200, 0), (30000, 1152, 384, 0),
                                            (5000, 192, 384, 64), (33, 4, 8, 0)])
def test_wgrad_bf16_register_staged(cuda, R, M, N, ld_extra):
    """asrx_wgrad_bf16 (csrc/gemm_wg.hip): dW += dY^T X over R rows, bf16 operands / fp32 accumulate,
    against float64 on the same bf16-rounded operands; accumulates into the existing dW; a column block
    of a wider dY (row stride > M) as wgrad_cols reads it."""
    from asrx import gemm as G, prec

    g = torch.Generator().manual_seed(R + M)
    dyw = torch.randn(R, M + ld_extra, generator=g)
    x = torch.randn(R, N, generator=g)
    w0 = torch.randn(M, N, generator=g)
    out = w0.clone().to(cuda)
    with prec.precision("bf16"):
        if ld_extra:
            G.wgrad_cols(dyw.to(cuda), ld_extra, M, x.to(cuda), out)
            dy = dyw[:, ld_extra:]
        else:
            G.linear_wgrad(dyw.to(cuda), x.to(cuda), out=out, accumulate=True)
            dy = dyw
    ref = w0.double() + _bf(dy).t() @ _bf(x)
    err = float((out.cpu().double() - ref).abs().max() / (_bf(dy).t().abs() @ _bf(x).abs()).max())
    assert err < 1e-5, err


@pytest.mark.parametrize("n", [12345, 16001, 480077, 160 * 3000])
def test_wave_pool_any_length(cuda, n):
    """asrx_wave_pool (adaptive_avg_pool1d to int(N/160) bins for any N, essentials.py:493-510) against
    the float64 oracle, and equal to the fused pool of the log-mel pass when 160 | N."""
    import numpy as np

    from asrx import mel
    from oracle import mel as omel

    g = torch.Generator().manual_seed(n)
    x = torch.randn(2, n, generator=g)
    T = n // 160
    got = mel.wave_pool(x.to(cuda), T).cpu()
    for b in range(2):
        ref = torch.from_numpy(omel.waveform_feature(x[b].numpy().astype(np.float64))[0])
        assert float((got[b].double() - ref).abs().max()) < 1e-6
    if n % 160 == 0:
        _, fused = mel.logmel(x.to(cuda), layout="BMF", pool=True)
        assert float((fused.cpu() - got).abs().max()) < 1e-6
