"""CPU restatement of MaxFactor.step (optimizerc.py:6-147) — TEST INFRASTRUCTURE ONLY (see
oracle/__init__.py).  PARITY UNPINNED: the reference ships no optimizer tests or fixtures and
executing it was denied; checked by review against the cited lines and by the
known-answer test in tests/test_oracle_maxfactor.py.

Operates on CPU float64 copies: ``params`` is a list of dicts {"p", "grad", "state", "group"} with the
group's hyper-parameters; the state dict uses the reference's names (step, row_var, col_var, v).
"""
from __future__ import annotations

import torch


def init_state(p: torch.Tensor) -> dict:
    """optimizerc.py:39-46 (state["RMS"] is written there but never read: omitted)."""
    st = {"step": 0.0, "v": torch.zeros_like(p)}
    if p.dim() > 1:
        rs, cs = list(p.shape), list(p.shape)
        rs[-1], cs[-2] = 1, 1
        st["row_var"], st["col_var"] = p.new_zeros(rs), p.new_zeros(cs)
    return st


def step_param(p: torch.Tensor, grad: torch.Tensor, st: dict, g: dict) -> None:
    """One parameter of one MaxFactor step, in place (optimizerc.py:55-133)."""
    eps1, eps2 = g["eps"]
    if g["max"]:  # :58-59
        grad = -grad
    st["step"] += 1  # :65
    t = st["step"]
    beta = t ** g["b_decay"]  # :69
    rho = max(g["min_lr"], min(g["lr"], 1.0 / (t ** 0.5)))  # :74
    alpha = max(eps2, float(p.norm(2)) / (p.numel() ** 0.5)) * rho  # :75
    if g["decay"] != 0:  # :77-78
        p.mul_(1 - g["lr"] * g["decay"])
    if grad.dim() > 1:  # :80-87
        row_mean = torch.norm(grad, dim=-1, keepdim=True).square_().div_(grad.size(-1) + 1e-8)
        st["row_var"].lerp_(row_mean, beta)
        col_mean = torch.norm(grad, dim=-2, keepdim=True).square_().div_(grad.size(-2) + 1e-8)
        st["col_var"].lerp_(col_mean, beta)
        var_est = st["row_var"] @ st["col_var"]
        max_row_var = st["row_var"].max(dim=-2, keepdim=True)[0]
        var_est.div_(max_row_var.clamp_(min=eps1))
    else:  # :88-90
        st["v"].mul_(g["gamma"]).add_(grad ** 2, alpha=1 - g["gamma"])
        var_est = st["v"]
    update = var_est.clamp_(min=eps1 * eps1).rsqrt_().mul_(grad)  # :92
    inf_norm = torch.norm(update, float("inf"))  # :95-97
    if inf_norm > 0:
        update.div_(inf_norm.clamp_(min=eps1))
    denom = max(1.0, float(update.norm(2)) / ((update.numel() ** 0.5) * g["d"]))  # :99
    if p.dim() < 3 or g["bias"] == 1:  # :111-116
        scale = update.abs().max(dim=-1, keepdim=True)[0]
    else:
        scale = torch.median(update.abs(), dim=-1, keepdim=True)[0]
    final_direction = update.sign() * scale
    step_size = alpha / denom  # :117
    p.add_(final_direction, alpha=-step_size)  # :128


def step(params: list) -> None:
    for e in params:
        if e["grad"] is None:
            continue
        step_param(e["p"], e["grad"], e["state"], e["group"])
