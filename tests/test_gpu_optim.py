"""Fused MaxFactor step (asrx/optim.py -> asrx_maxfactor_step) against the CPU restatement
(oracle/maxfactor.py of optimizerc.py:6-147) over several steps: vectors, matrices, 3-D conv
weights, the bias=2 group's median path, parameters without gradients, and the reference's two
parameter groups / hyper-parameters (model.py:772-787)."""
import pytest
import torch

from oracle import maxfactor as omf

pytestmark = pytest.mark.gpu

SHAPES = [((37, 53), 0), ((16, 4, 3), 0), ((29,), 0), ((), 0), ((384, 1, 1), 0), ((300, 40), 0),
          ((1, 1, 384), 1), ((8, 20), 1), ((5,), 1), ((6, 2, 10), 1),
          # short rows packed several to a wave (lane groups of 4 / 16 / 32), ragged last work item
          ((48, 40, 3), 1), ((7, 5, 15), 0), ((33, 17), 0), ((9, 7, 2), 1)]


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("steps", [4])
def test_maxfactor_matches_oracle(cuda, steps):
    from asrx.optim import MaxFactor

    torch.manual_seed(0)
    params = [torch.randn(s, dtype=torch.float32) for s, _ in SHAPES]
    dev = [p.to(cuda).requires_grad_(True) for p in params]
    ref = [p.double().clone() for p in params]
    hp = dict(lr=2.5e-3, b_decay=-0.8, eps=(1e-8, 1e-8), d=1.0, decay=1e-2, gamma=0.99, max=False, bias=1,
              min_lr=1e-9, clip=False, cap=0.0)
    groups = [{"params": [d for d, (_, gi) in zip(dev, SHAPES) if gi == 0], "bias": 1.0},
              {"params": [d for d, (_, gi) in zip(dev, SHAPES) if gi == 1], "bias": 2.0}]
    opt = MaxFactor(groups, **hp)
    states = [omf.init_state(r) for r in ref]
    gen = torch.Generator().manual_seed(1)
    for it in range(steps):
        grads = [torch.randn(s, generator=gen) * (0.1 + 3 * i) for i, (s, _) in enumerate(SHAPES)]
        for i, (d, g) in enumerate(zip(dev, grads)):
            d.grad = None if (it == 1 and i == 2) else g.to(cuda)  # a step without a gradient
        opt.step()
        for i, (r, g, (_, gi)) in enumerate(zip(ref, grads, SHAPES)):
            if it == 1 and i == 2:
                continue
            omf.step_param(r, g.double(), states[i], dict(hp, bias=1.0 if gi == 0 else 2.0))
        torch.cuda.synchronize()
        for i, (d, r) in enumerate(zip(dev, ref)):
            assert _rel(d, r) < 2e-6, (it, SHAPES[i], _rel(d, r))
    for i, d in enumerate(dev):
        st = opt.state[d]
        if d.dim() > 1:
            assert _rel(st["row_var"], states[i]["row_var"]) < 1e-5
            assert _rel(st["col_var"], states[i]["col_var"]) < 1e-5
        else:
            assert _rel(st["v"], states[i]["v"]) < 1e-5


def test_maxfactor_reference_groups_on_model(cuda):
    """The reference's grouping over the real module tree steps every parameter with a gradient."""
    from asrx.config import Dimensions
    from asrx.model import Model
    from asrx.optim import FAMScheduler2, MaxFactor, reference_param_groups

    torch.manual_seed(0)
    m = Model(Dimensions(tokens=300, mels=128, dims=128, head=2, layer=4, act="gelu", n_type="AbbyNormal")).to(cuda)
    groups = reference_param_groups(m)
    assert sum(len(g["params"]) for g in groups) == sum(1 for p in m.parameters() if p.requires_grad)
    opt = MaxFactor(groups, lr=2.5e-3, b_decay=-0.8, eps=(1e-8, 1e-8), d=1.0, decay=1e-2, gamma=0.99, max=False,
                    bias=1, min_lr=1e-9, clip=False, cap=0.0)
    sched = FAMScheduler2(opt, warmup_steps=10, total_steps=100, decay_start=None, warmup_start=1e-6, eta_min=1e-6)
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    sched.step()
    torch.cuda.synchronize()
    for n, p in m.named_parameters():
        assert torch.isfinite(p).all(), n
        assert torch.equal(p, before[n]) != p.requires_grad, n  # frozen ones (v_gate.tx) untouched
    assert abs(opt.param_groups[0]["lr"] - (1e-6 + (2.5e-3 - 1e-6) * 0.1)) < 1e-12
