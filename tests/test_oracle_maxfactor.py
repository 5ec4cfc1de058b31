"""Known-answer checks of the MaxFactor restatement (oracle/maxfactor.py) on CPU."""
import math

import torch

from oracle import maxfactor as omf

G = dict(lr=2.5e-3, b_decay=-0.8, eps=(1e-8, 1e-8), d=1.0, decay=1e-2, gamma=0.99, max=False, bias=1.0,
         min_lr=1e-9, clip=False, cap=0.0)


def test_vector_first_step_is_a_sign_step():
    """1-D parameter, step 1: v = 0.01 g^2, u = g / |g| * 10 -> normalised to sign(g); the max over
    the vector is 1, so p <- p (1 - lr decay) - alpha / denom * sign(g) with alpha = rms(p) * lr and
    denom = max(1, ||sign g|| / sqrt(n)) = 1."""
    torch.manual_seed(0)
    p = torch.randn(17, dtype=torch.float64)
    g = torch.randn(17, dtype=torch.float64)
    expect = p * (1 - G["lr"] * G["decay"]) - (p.norm() / math.sqrt(17)) * G["lr"] * g.sign()
    st = omf.init_state(p)
    omf.step_param(p, g, st, G)
    assert torch.allclose(p, expect, rtol=0, atol=1e-12)
    # optimizerc.py:89-97 works in place on var_est, which for a vector IS state["v"]: after the
    # step v holds the normalised update (here sign(g)), and the next step's EMA starts from that
    assert torch.allclose(st["v"], g.sign())


def test_matrix_state_is_factored_and_median_group():
    torch.manual_seed(1)
    p = torch.randn(1, 1, 9, dtype=torch.float64)  # like jump.mem_w: 3-D in the bias=2 group -> median
    g = torch.randn(1, 1, 9, dtype=torch.float64)
    st = omf.init_state(p)
    assert st["row_var"].shape == (1, 1, 1) and st["col_var"].shape == (1, 1, 9)
    q = p.clone()
    omf.step_param(q, g, st, dict(G, bias=2.0))
    d = (p * (1 - G["lr"] * G["decay"]) - q)
    # every element moved by the same magnitude (the row's median |u|), in the direction of g
    assert torch.allclose(d.abs(), d.abs().max().expand_as(d))
    assert torch.equal(torch.sign(d), torch.sign(g))
