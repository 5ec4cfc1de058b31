"""Plain bf16 products on the vendor library (asrx_gemm_lt, hipBLASLt; csrc/gemm_lt.cpp) -- the shapes asrx/gemm.py
routes there (bf16 activations, K >= 768, >= 16384 rows; model.py:573-574, 505 and their input gradients): against a
float64 product of the same bf16 operands within fp32 accumulation error, against the hand-written wide GEMM on the
same operands (LIBRARY_GEMM off) within the same bound, with bias, alpha / beta accumulation and bf16 output, and
repeat launches bit-identical (the step's forward must stay deterministic)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


@pytest.mark.parametrize("M,N,K", [(48016, 768, 768), (192064, 384, 1152), (24000, 1024, 3072), (16384, 200, 776)])
@pytest.mark.parametrize("cbf,beta,bias", [(False, 0.0, True), (False, 1.0, False), (True, 0.0, True)])
def test_library_gemm_matches_reference_and_wide(cuda, M, N, K, cbf, beta, bias):
    from asrx import gemm as G
    from asrx import prec

    g = torch.Generator().manual_seed(M + N + K + 3 * cbf + int(beta))
    A = torch.randn(M, K, generator=g).to(cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda) if bias else None
    C0 = torch.randn(M, N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    dt = torch.bfloat16 if cbf else torch.float32
    with prec.precision("bf16"):
        assert G._lib_ok(A, Wb, C0.to(dt), M, N, K, K, N, None, "none", False, None, beta)

        def run(lib_on):
            old = G.LIBRARY_GEMM
            G.LIBRARY_GEMM = lib_on
            try:
                C = C0.clone().to(dt)
                G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N, bias=b, beta=beta)
                return C
            finally:
                G.LIBRARY_GEMM = old
        lt, lt2, wide = run(True), run(True), run(False)
    torch.cuda.synchronize()
    assert torch.equal(lt, lt2)  # deterministic
    ref = A.double() @ Wb.view(torch.bfloat16).double().t() + (b.double() if bias else 0.0) + beta * C0.double()
    tol = 1e-2 if cbf else 1e-5  # bf16 output: one rounding of the result
    assert _rel(lt, ref) < tol, _rel(lt, ref)
    assert _rel(wide, ref) < tol
    assert _rel(lt, wide) < 2 * tol


def test_library_gemm_not_used_for_fused_or_small_products(cuda):
    """K = 384, fp32 activations, activations / saved pre-activations, row-tile lists and the 8192-row text side keep
    the hand-written kernels (the library only measured faster for plain products at K >= 768, >= 16384 rows)."""
    from asrx import gemm as G

    A16 = torch.zeros(32768, 1152, device=cuda, dtype=torch.bfloat16)
    W = G.weight_bf16(torch.zeros(384, 1152, device=cuda), cache=False)
    C = torch.zeros(32768, 384, device=cuda)
    assert G._lib_ok(A16, W, C, 32768, 384, 1152, 1152, 384, None, "none", False, None, 0.0)
    assert not G._lib_ok(A16.float(), W, C, 32768, 384, 1152, 1152, 384, None, "none", False, None, 0.0)
    assert not G._lib_ok(A16, W, C, 32768, 384, 1152, 1152, 384, None, "gelu", False, None, 0.0)
    assert not G._lib_ok(A16, W, C, 32768, 384, 1152, 1152, 384, C, "none", False, None, 0.0)
    assert not G._lib_ok(A16[:8192], W, C[:8192], 8192, 384, 1152, 1152, 384, None, "none", False, None, 0.0)
    A3 = torch.zeros(32768, 384, device=cuda, dtype=torch.bfloat16)
    W3 = G.weight_bf16(torch.zeros(384, 384, device=cuda), cache=False)
    assert not G._lib_ok(A3, W3, C, 32768, 384, 384, 384, 384, None, "none", False, None, 0.0)
