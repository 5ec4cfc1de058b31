"""MSheath.forward without a backward issued from C++ in one call (asrx_msheath_fwd, csrc/msheath_plan.cpp) against
the Python loop that issues the same launches one by one (asrx/msheath.py forward(save=False); model.py:429-507):
the same kernels with the same arguments, so the outputs are BIT-IDENTICAL -- over widths of every row-kernel
instantiation, one and several samples, sequences shorter than a GEMM tile, and policy noise that sends samples
through different layer trajectories (the row-tile lists of partially active layers)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,B,L,seed", [(384, 2, 3001, 1), (384, 5, 256, 2), (384, 3, 77, 3), (128, 4, 300, 4),
                                        (768, 2, 500, 5), (1024, 2, 301, 6), (512, 3, 129, 7)])
def test_msheath_composite_matches_python_loop(cuda, D, B, L, seed):
    from asrx import gemm as G
    from asrx import msheath, ops, prec
    from asrx.model import MSheath

    torch.manual_seed(seed)
    mod = MSheath(D, max(D // 64, 1), 4).cuda()
    x = torch.randn(B, L, D, device=cuda)
    outs = []
    try:
        with prec.precision("bf16"), torch.no_grad():
            for key in (11 * seed, 11 * seed + 1, 11 * seed + 2):
                gpol = ops.policy_noise(B, len(mod.layers), 0, key, cuda)
                for comp in (False, True):
                    msheath.COMPOSITE = comp
                    outs.append(msheath.msheath(mod, x, gpol).clone())
    finally:
        msheath.COMPOSITE = True
        G.end_step()
    torch.cuda.synchronize()
    for k in range(0, len(outs), 2):
        assert torch.isfinite(outs[k]).all()
        assert torch.equal(outs[k + 1], outs[k]), (k, float((outs[k + 1] - outs[k]).abs().max()))


def test_msheath_composite_not_used_outside_bf16(cuda):
    """fp32 parity mode (and a probed or decision-recording run) keeps the Python loop: the composite covers the wide
    bf16-weight GEMM only."""
    from asrx import gemm as G
    from asrx import msheath, ops, prec
    from asrx.model import MSheath

    mod = MSheath(384, 6, 2).cuda()
    x = torch.randn(2, 100, 384, device=cuda)
    gpol = ops.policy_noise(2, 2, 0, 5, cuda)
    with prec.precision("fp32"):
        assert not msheath._composite_ok(mod, x, gpol, None)
    with prec.precision("bf16"):
        assert msheath._composite_ok(mod, x, gpol, None)
        assert not msheath._composite_ok(mod, x, gpol[:, :1], None) or gpol[:, :1].is_contiguous()
    G.end_step()
