"""Repeat-launch stress of the wide-GEMM kernels whose LDS regions are shared by all eight waves (VERDICT r05 item 5:
a round-5 experiment -- the AbbyNormal router on gemm_ws with W2 staged in LDS -- gave transiently wrong partials).
A missing barrier between the resident weight-slice fill, the activation images and the epilogue slabs shows up as
an output that changes from launch to launch on the same inputs.  Each kernel runs REPEATS times at the router /
projection shape (192064 x 384 x 384, the step's largest K = 384 products) and at a ragged shape, and every
launch must equal the first bit for bit and equal the other kernels (the three are bit-identical by construction):
gemm_ws_kernel (variant 13), gemm_p2_kernel (1), gemm_wr_kernel (0), with the epilogues the step uses (bias,
activation, saved pre-activation, residual, rotary), bf16 and fp32 activations, and the AbbyNormal router
epilogue (gemm_wr_kernel's w2s / red LDS regions, router64_kernel at d = 64).  The LDS audit: DESIGN.md §7."""
import pytest
import torch

pytestmark = pytest.mark.gpu

REPEATS = 24


def _variant(v, fn):
    from asrx import lib

    old = lib.load().asrx_set_gemm_variant(v)
    try:
        return fn()
    finally:
        lib.load().asrx_set_gemm_variant(old)


@pytest.mark.parametrize("M", [192064, 48017])
@pytest.mark.parametrize("abf", [False, True])
@pytest.mark.parametrize("act,res", [("none", False), ("silu", False), ("none", True)])
def test_wide_gemm_repeat_launches_identical(cuda, M, abf, act, res):
    from asrx import gemm as G
    from asrx import lib

    N = K = 384
    g = torch.Generator().manual_seed(M + 3 * abf + 5 * res)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    xa = x.to(torch.bfloat16) if abf else x
    if res and abf:
        pytest.skip("the residual epilogue takes fp32 activations (the out projection)")

    def once():
        y = torch.empty(M, N, device=cuda)
        if res:
            lib.call("asrx_gemm_wn_res", lib.ptr(xa), K, lib.ptr(Wb), K, lib.ptr(y), N, lib.ptr(b), lib.ptr(R), N, M, N,
                     K, 3, lib.stream())
            return (y,)
        z = torch.empty(M, N, device=cuda)
        G.gemm_wn(xa, Wb, y, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act=act, Z=z)
        return y, z

    outs = {}
    for v in (13, 1, 0):
        def rep():
            first = once()
            bad = 0
            for _ in range(REPEATS - 1):
                again = once()
                bad += int(not all(torch.equal(a, c) for a, c in zip(first, again)))
            return first, bad
        outs[v] = _variant(v, rep)
    torch.cuda.synchronize()
    for v, (_, bad) in outs.items():
        assert bad == 0, f"variant {v}: {bad} of {REPEATS - 1} repeat launches differed"
    for v in (1, 0):
        assert all(torch.equal(a, c) for a, c in zip(outs[13][0], outs[v][0])), v


@pytest.mark.parametrize("M,d", [(192064, 384), (96000, 384), (1152384, 64)])
@pytest.mark.parametrize("keep", [True, False])
def test_router_repeat_launches_identical(cuda, M, d, keep):
    """The AbbyNormal router (essentials.py:155-161) on gemm_wr_kernel's router epilogue (W2 in LDS `w2s`, per-wave
    row partials through LDS `red`, s_barrier merge) and on router64_kernel: REPEATS launches bit-identical."""
    from asrx import gemm as G

    g = torch.Generator().manual_seed(M + d + keep)
    x = torch.randn(M, d, generator=g).to(cuda)
    W1 = (torch.randn(d, d, generator=g) / d ** 0.5).to(cuda)
    b1 = torch.randn(d, generator=g).to(cuda)
    W2 = (torch.randn(3, d, generator=g) / d ** 0.5).to(cuda)
    first = G.router_fwd(x, W1, b1, W2, keep)
    bad = 0
    for _ in range(REPEATS - 1):
        h, lg = G.router_fwd(x, W1, b1, W2, keep)
        bad += int(not torch.equal(lg, first[1]) or (keep and not torch.equal(h, first[0])))
    torch.cuda.synchronize()
    assert bad == 0, bad
    G.end_step()
