"""CPU: which bf16 rounding points make the perf-mode gradient unreliable (VERDICT r03 missing 1).
The float64 oracle is re-run with its operands rounded to bf16 at chosen points (oracle/model.py EMU,
straight-through), decisions replayed from the pure float64 run, and its gradient compared with the
pure float64 gradient (whole-gradient cosine, worst parameter).  usage:
  bf16_sensitivity.py B seconds T [cfg] point[,point...] ...
points: lin (every Linear's operands but q/kv), qkproj (the q / kv projections' operands), qk (the
attention's q, k), pv (softmax P and v), logits (the tied logits' operands); modifiers: x3 (operands as a
split-bf16 hi + lo pair instead of one bf16), nudgeE (no rounding: weights nudged by relative 2^-E)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from oracle import model as om  # noqa: E402

B, sec, T = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
cfg = CONFIGS[sys.argv[4]]
sets = [a.split(",") for a in sys.argv[5:]]
torch.manual_seed(0)
sd = {k: v.detach() for k, v in Model(cfg).state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, 0)
ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}
rec = om.Decisions()
t0 = time.time()
P0, r0 = mp.oracle_run(sd, ocfg, x, rec, torch.float64)
print(f"float64 reference run {time.time() - t0:.1f}s loss {r0['loss']:.6f}", flush=True)
def nudged(sd, seed, rel):
    g = torch.Generator().manual_seed(1000 + seed)
    return {k: (v.detach().double() * (1 + (torch.rand(v.shape, generator=g, dtype=torch.float64) * 2 - 1) * rel)
                if v.is_floating_point() else v) for k, v in sd.items()}


for pts in sets:
    om.EMU.clear()
    # "nudgeE": no rounding, weights nudged by relative 2^-E uniform noise (E = 9: bf16 resolution; 17: the
    # resolution of a split-bf16 hi + lo pair; 24: one fp32 ulp)
    nud = [int(p[5:]) for p in pts if p.startswith("nudge")]
    om.EMU.update(p for p in pts if p != "none" and not p.startswith("nudge"))
    t0 = time.time()
    src = nudged(sd, 0, 2.0 ** -nud[0]) if nud else sd
    Pk, rk = mp.oracle_run(src, ocfg, x, om.Decisions(table=rec.rec), torch.float64)
    om.EMU.clear()
    d = mp.grad_distance(Pk, P0)
    lg = float((rk["logits"] - r0["logits"]).abs().max() / r0["logits"].abs().max())
    print(f"bf16 at {'+'.join(pts):24s} loss rel {abs(rk['loss'] - r0['loss']) / abs(r0['loss']):.2e}  logits "
          f"{lg:.2e}  grads global {d[0]:.3e} ({d[1]})  cos {d[2]:.5f}  [{time.time() - t0:.0f}s]", flush=True)

# per parameter: cosine of the all-points bf16 emulation's gradient with float64, and of float64 on weights
# nudged at bf16 scale (relative 2^-9 uniform noise) -- the gradient field's roughness at bf16 resolution
if os.environ.get("PER_PARAM"):
    def nudge(sd, seed, rel):
        g = torch.Generator().manual_seed(1000 + seed)
        return {k: (v.detach().double() * (1 + (torch.rand(v.shape, generator=g, dtype=torch.float64) * 2 - 1) * rel)
                    if v.is_floating_point() else v) for k, v in sd.items()}

    om.EMU.update(["lin", "qkproj", "qk", "pv", "logits"])
    Pe, _ = mp.oracle_run(sd, ocfg, x, om.Decisions(table=rec.rec), torch.float64)
    om.EMU.clear()
    Pn, _ = mp.oracle_run(nudge(sd, 0, 2.0 ** -9), ocfg, x, om.Decisions(table=rec.rec), torch.float64)
    print(f"weights nudged at bf16 scale: {mp.grad_distance(Pn, P0)}")
    names = [n for n in P0 if torch.is_tensor(P0[n]) and P0[n].grad is not None
             and not any(z in n for z in mp.ANALYTIC_ZERO)]
    rows = []
    for n in names:
        g0 = P0[n].grad.double().reshape(-1)
        c = lambda a: float((a @ g0) / (a.norm() * g0.norm()).clamp_min(1e-300))  # noqa: E731
        rows.append((c(Pe[n].grad.double().reshape(-1)), c(Pn[n].grad.double().reshape(-1)), n,
                     float(g0.abs().max())))
    rows.sort()
    for ce, cn, n, gm in rows:
        print(f"  {ce:9.5f} {cn:9.5f}  {gm:10.3e}  {n}")
