"""Split-bf16 ("x3") products in the generic GEMM (csrc/gemm.hip PREC_X3): x = bf16 hi + bf16 lo and
hi*hi + hi*lo + lo*hi on the bf16 MFMA.  Against float64 on random operands its error must sit at the
~16-bit operand level -- two orders below one bf16 rounding (PREC_BF16) and close to exact fp32 (PREC_F32) --
for every operand layout the model uses (forward, input gradient, weight gradient with split-K, k3 conv)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _err(c, ref):
    return float((c.double() - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("M,N,K", [(1000, 384, 384), (260, 200, 96), (4096, 1536, 1152)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (False, True), (True, False), (False, False)])
def test_x3_gemm_precision(cuda, M, N, K, a_kc, b_kc):
    from asrx import gemm as G
    from asrx import prec

    g = torch.Generator().manual_seed(M + N + K + 2 * a_kc + b_kc)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(K, N, generator=g, dtype=torch.float64) / K ** 0.5
    ref = A @ Bm
    Ad = (A if a_kc else A.t()).contiguous().float().to(cuda)  # K-contiguous: (M, K); else stored (K, M) (leading dims: multiples of 4)
    Bd = (Bm.t() if b_kc else Bm).contiguous().float().to(cuda)  # K-contiguous: stored (N, K); else (K, N)
    out = {}
    for p in (prec.PREC_X3, prec.PREC_BF16, prec.PREC_F32):
        C = torch.empty(M, N, device=cuda)
        G.gemm(Ad, Bd, C, M=M, N=N, K=K, lda=Ad.shape[1], ldb=Bd.shape[1], ldc=N, a_kc=a_kc, b_kc=b_kc,
               precision=p)
        out[p] = _err(C.cpu(), ref)
    print(M, N, K, a_kc, b_kc, {"x3": out[prec.PREC_X3], "bf16": out[prec.PREC_BF16], "fp32": out[prec.PREC_F32]})
    assert out[prec.PREC_X3] < 5e-5
    assert out[prec.PREC_X3] < out[prec.PREC_BF16] / 50
    assert out[prec.PREC_X3] < 50 * max(out[prec.PREC_F32], 1e-7)


def test_x3_splitk_and_conv(cuda):
    from asrx import gemm as G
    from asrx import prec

    g = torch.Generator().manual_seed(1)
    rows, M, K = 20000, 384, 384  # weight gradient: out (M, K) += A^T X over rows, split-K
    A = torch.randn(rows, M, generator=g, dtype=torch.float64)
    X = torch.randn(rows, K, generator=g, dtype=torch.float64)
    ref = A.t() @ X
    out = torch.zeros(M, K, device=cuda)
    G.gemm(A.float().to(cuda), X.float().to(cuda), out, M=M, N=K, K=rows, lda=M, ldb=K, ldc=K, a_kc=False,
           b_kc=False, beta=1.0, splitk=8, precision=prec.PREC_X3)
    assert _err(out.cpu(), ref) < 5e-5
    # k3 conv (implicit im2col, channels-last, padding 1) forward
    Bn, T, C, O = 2, 301, 128, 384
    x = torch.randn(Bn, T, C, generator=g, dtype=torch.float64)
    W = torch.randn(O, 3 * C, generator=g, dtype=torch.float64) / (3 * C) ** 0.5
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1))
    col = torch.cat([xp[:, k:k + T] for k in range(3)], -1)  # (B, T, 3C), tap-major like the kernel's K order
    ref = col @ W.t()
    y = torch.empty(Bn, T, O, device=cuda)
    G.gemm(x.float().to(cuda), W.float().to(cuda), y, M=Bn * T, N=O, K=3 * C, lda=C, ldb=3 * C, ldc=O, a_kc=True,
           b_kc=True, conv_a=True, conv_F=T, conv_C=C, precision=prec.PREC_X3)
    assert _err(y.cpu(), ref) < 5e-5
