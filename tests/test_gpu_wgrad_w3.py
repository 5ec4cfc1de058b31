"""The wide weight-gradient work items (csrc/gemm_wg.hip wgrad_w3_kernel: 128 dY features x 384 X features,
asrx_set_wgrad_variant(1), the default for fp32 dY with bf16-stored X, N % 384 == 0 and >= 8 such items per
K slice; the 384 x 384 case stays on the 128 x 128 items either way) against the 128 x 128
items of wgrad_wr_kernel (variant 0): dW += dY^T X and db += column sums of dY (the backward of every
Linear on a bf16-stored input, model.py:242-245, 421-425, 573-574).  Both sum K slices with float atomics, so
they agree to fp32 reassociation; both equal a float64 product of the bf16-rounded operands within
accumulation error -- for ragged row counts, feature counts that are not multiples of 128, and the bias."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dy, xb, M, N, R, db):
    from asrx import lib

    out = torch.zeros(M, N, device=dy.device)
    dbo = torch.zeros(M, device=dy.device) if db else None
    if db:
        lib.call("asrx_wgrad_bias", lib.ptr(dy), 0, M, lib.ptr(xb), 1, N, lib.ptr(out), N, lib.ptr(dbo), M, N, R,
                 8, lib.stream())
    else:
        lib.call("asrx_wgrad_bf16_ex", lib.ptr(dy), M, lib.ptr(xb), 1, N, lib.ptr(out), N, M, N, R, 8, lib.stream())
    return out, dbo


@pytest.mark.parametrize("M,N,R", [(1536, 384, 192064), (1536, 384, 50001), (1152, 384, 9000), (384, 1536, 30000),
                                   (256, 1536, 4096), (384, 384, 20000)])
@pytest.mark.parametrize("db", [False, True])
def test_wgrad_w3_matches(cuda, M, N, R, db):
    from asrx import lib

    g = torch.Generator().manual_seed(M + N + R + db)
    dy = torch.randn(R, M, generator=g).to(cuda)
    x = torch.randn(R, N, generator=g).to(cuda)
    xb = x.to(torch.bfloat16)
    old = lib.load().asrx_set_wgrad_variant(1)
    try:
        w1, d1 = _run(dy, xb, M, N, R, db)
        lib.load().asrx_set_wgrad_variant(0)
        w0, d0 = _run(dy, xb, M, N, R, db)
    finally:
        lib.load().asrx_set_wgrad_variant(old)
    scale = float(w0.abs().max())
    assert float((w1 - w0).abs().max()) <= 1e-5 * scale
    ref = dy.to(torch.bfloat16).double().t() @ xb.double()
    assert float((w1.double() - ref).abs().max() / ref.abs().max()) < 1e-5
    if db:
        refb = dy.double().sum(0)
        assert float((d1.double() - refb).abs().max()) <= 1e-5 * float(dy.abs().sum(0).max())
        assert float((d1 - d0).abs().max()) <= 1e-5 * float(dy.abs().sum(0).max())
