"""Gradient diagnostics of the bf16 perf mode: per-op bf16 gradients against float64 autograd, and the
whole model's bf16 gradients against its fp32 parity-mode gradients, parameter by parameter.

python tools/grad_diag.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from asrx import ops, prec  # noqa: E402
from asrx.config import CONFIGS, Dimensions  # noqa: E402
from asrx.model import AbbyNormal, Model  # noqa: E402
from oracle import keys as K  # noqa: E402
from oracle import model as om  # noqa: E402
import model_parity as mp  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def op_abby(d, H=1, precision="bf16"):
    torch.manual_seed(0)
    mod = AbbyNormal(d).cuda()
    B, L = 2, 301
    x = torch.randn(B, L, H, d) * 3.0 if H > 1 else torch.randn(B, L, d) * 3.0
    P = {f"n.{k}": v.detach().cpu() for k, v in mod.state_dict().items()}
    seed, step, site, sid_base = 5, 2, "t.abby", 3
    key = K.site_key(seed, step, site)
    noise = om.Noise(seed, step, torch.float64)
    sids = [sid_base + b for b in range(B)]
    r = mod.mode_router
    ins = [x, r[0].weight.detach().cpu(), r[0].bias.detach().cpu(), r[2].weight.detach().cpu(),
           r[2].bias.detach().cpu()]
    g_in = [t.detach().cuda().requires_grad_(True) for t in ins]
    r_in = [t.detach().double().requires_grad_(True) for t in ins]
    with prec.precision(precision):
        yg = ops.AbbyNormalFn.apply(*g_in, L, H, sid_base, key, True, True)
    PP = dict(P)
    PP.update({"n.mode_router.0.weight": r_in[1], "n.mode_router.0.bias": r_in[2], "n.mode_router.2.weight": r_in[3],
               "n.mode_router.2.bias": r_in[4]})
    g = noise.abby(site, sids, H, L)
    g = g.permute(0, 2, 1, 3) if H > 1 else g[:, 0]
    yr = om.abby_normal(PP, "n", r_in[0], g)
    gout = torch.randn(yr.shape, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    with prec.precision(precision):
        yg.backward(gout.float().cuda())
    yr.backward(gout)
    return {"op": f"abby d={d} H={H} {precision}", "y": rel(yg, yr),
            "grads": [rel(a.grad, b.grad) for a, b in zip(g_in, r_in)]}


def op_linear(M, K_, N, act, precision="bf16"):
    g = torch.Generator().manual_seed(1)
    x, W, b = torch.randn(M, K_, generator=g), torch.randn(N, K_, generator=g) / K_ ** 0.5, torch.randn(N, generator=g)
    gi = [t.cuda().requires_grad_(True) for t in (x, W, b)]
    ri = [t.double().requires_grad_(True) for t in (x, W, b)]
    with prec.precision(precision):
        yg = ops.linear(gi[0], gi[1], gi[2], act=act)
    yr = F.linear(ri[0], ri[1], ri[2])
    yr = {"none": yr, "gelu": F.gelu(yr), "silu": F.silu(yr), "sigmoid": torch.sigmoid(yr)}[act]
    gout = torch.randn(yr.shape, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    with prec.precision(precision):
        yg.backward(gout.float().cuda())
    yr.backward(gout)
    return {"op": f"linear {M}x{K_}x{N} {act} {precision}", "y": rel(yg, yr),
            "grads": [rel(a.grad, b.grad) for a, b in zip(gi, ri)]}


def model_grads(cfgname="tiny", B=1, seconds=3.0, T=32):
    cfg = CONFIGS[cfgname]
    x = mp.inputs(B, seconds, T, cfg.tokens)
    res = {}
    for precision in ("fp32", "bf16"):
        torch.manual_seed(0)
        m = Model(cfg).cuda().train()
        m.set_noise(7, 3)
        with prec.precision(precision):
            out = m(labels=x["labels"].cuda(), text_ids=x["text_ids"].cuda(), spectrogram=x["spectrogram"].cuda(),
                    pitch=x["pitch"].cuda(), waveform=x["waveform"].cuda())
            out["loss"].backward()
        res[precision] = ({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None},
                          out["logits"].detach(), float(out["loss"]))
    g32, l32, lo32 = res["fp32"]
    g16, l16, lo16 = res["bf16"]
    rows = sorted(((rel(g16[n], g32[n]), n, float(g32[n].abs().max()), float(g16[n].abs().max())) for n in g32),
                  reverse=True)
    return {"model": cfgname, "logits": rel(l16, l32), "argmax": float((l16.argmax(-1) == l32.argmax(-1)).double().mean()),
            "loss": (lo32, lo16), "worst": rows[:25], "n": len(rows)}


_DEC = None  # when a list: AbbyNormal decisions (idx per row) of every call, in call order


def _run(cfg, x, attn_fp32=False, no_wide=False, precision="bf16", perturb=0.0):
    from asrx import gemm as G

    if perturb:
        g = torch.Generator().manual_seed(99)
        x = dict(x)
        x["spectrogram"] = x["spectrogram"] * (1 + perturb * torch.randn(x["spectrogram"].shape, generator=g))

    orig_attn, orig_wide = ops.attention, G.use_wide
    if attn_fp32:
        def attn32(q, k, v, causal):
            with prec.precision("fp32"):
                return ops.AttentionFn.apply(q, k, v, causal)
        ops.attention = attn32
    if no_wide:
        G.use_wide = lambda K: False
    try:
        torch.manual_seed(0)
        m = Model(cfg).cuda().train()
        m.set_noise(7, 3)
        with prec.precision(precision):
            out = m(labels=x["labels"].cuda(), text_ids=x["text_ids"].cuda(), spectrogram=x["spectrogram"].cuda(),
                    pitch=x["pitch"].cuda(), waveform=x["waveform"].cuda())
            out["loss"].backward()
    finally:
        ops.attention, G.use_wide = orig_attn, orig_wide
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}, out["logits"].detach()


def _record_abby():
    orig = ops.AbbyNormalFn.forward

    def fwd(ctx, *a):
        out = orig(ctx, *a)
        if _DEC is not None and torch.is_grad_enabled():
            _DEC.append(ctx.saved_tensors[5].detach().clone())
        return out
    ops.AbbyNormalFn.forward = staticmethod(fwd)


def variants(cfgname="tiny", B=1, seconds=3.0, T=32):
    global _DEC
    cfg = CONFIGS[cfgname]
    x = mp.inputs(B, seconds, T, cfg.tokens)
    _DEC = []
    g32, l32 = _run(cfg, x, precision="fp32")
    d32, _DEC = _DEC, None
    for name, kw in (("fp32+perturb1e-6", {"precision": "fp32", "perturb": 1e-6}),
                     ("fp32+perturb1e-4", {"precision": "fp32", "perturb": 1e-4}), ("bf16", {}),
                     ("bf16+attn32", {"attn_fp32": True}), ("bf16+nowide", {"no_wide": True}),
                     ("bf16+attn32+nowide", {"attn_fp32": True, "no_wide": True})):
        _DEC = []
        g, l = _run(cfg, x, **kw)
        dd, _DEC = _DEC, None
        flips = sum(int((a != b).sum()) for a, b in zip(d32, dd)) if len(dd) == len(d32) else -1
        rows = sum(a.numel() for a in d32)
        errs = sorted(((rel(g[n], g32[n]), n) for n in g32), reverse=True)
        med = errs[len(errs) // 2][0]
        print(json.dumps({"variant": name, "model": cfgname, "abby_flips": flips, "abby_rows": rows,
                          "logits": rel(l, l32),
                          "argmax": float((l.argmax(-1) == l32.argmax(-1)).double().mean()),
                          "median_grad": med, "worst": errs[:6]}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "variants":
        _record_abby()
        variants()
        variants("medium", 1, 2.0, 32)
        sys.exit(0)
    for d, H in ((384, 1), (64, 6), (128, 1)):
        for p in ("fp32", "bf16"):
            print(json.dumps(op_abby(d, H, p)), flush=True)
    for act in ("none", "gelu", "silu"):
        print(json.dumps(op_linear(3001, 384, 1152, act)), flush=True)
    print(json.dumps(op_linear(3001, 1152, 384, "none")), flush=True)
    print(json.dumps(model_grads()), flush=True)
