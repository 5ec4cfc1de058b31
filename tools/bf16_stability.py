"""CPU: per parameter, the relative L2 move of the float64 oracle's gradient under bf16-resolution
perturbations on one replayed trajectory -- operands rounded to bf16 in the forward (fwd), plus the
backward's arriving gradients (fwdbwd), and weights nudged by 2^-9 (nudge0/1) -- sorted, most stable first.
A parameter moved <= 10 % by all of them is "stable at bf16 resolution" (tests/test_gpu_model_configs.py).
usage: bf16_stability.py CONFIG B seconds T"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]
import torch
import model_parity as mp
from asrx.config import CONFIGS
from asrx.model import Model
from oracle import model as om
name=sys.argv[1]; B,sec,T=int(sys.argv[2]),float(sys.argv[3]),int(sys.argv[4])
cfg=CONFIGS[name]
torch.manual_seed(0)
sd = {k: v.detach() for k, v in Model(cfg).state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, 0)
ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}
rec = om.Decisions()
P0, r0 = mp.oracle_run(sd, ocfg, x, rec, torch.float64)
runs = {}
for tag, pts in (("fwd", mp.BF16_POINTS), ("fwdbwd", mp.BF16_POINTS + ("bwd",))):
    om.EMU.update(pts)
    runs[tag] = mp.oracle_run(sd, ocfg, x, om.Decisions(table=rec.rec), torch.float64)[0]
    om.EMU.clear()
runs["nudge0"] = mp.oracle_run(mp.bf16_nudge(sd, 0), ocfg, x, om.Decisions(table=rec.rec), torch.float64)[0]
runs["nudge1"] = mp.oracle_run(mp.bf16_nudge(sd, 1), ocfg, x, om.Decisions(table=rec.rec), torch.float64)[0]
names = [n for n in P0 if torch.is_tensor(P0[n]) and P0[n].grad is not None and not any(z in n for z in mp.ANALYTIC_ZERO)]
rows=[]
for n in names:
    g=P0[n].grad.reshape(-1)
    if float(g.abs().max()) == 0.0:
        continue
    rel={t: float((R[n].grad.reshape(-1)-g).norm()/g.norm().clamp_min(1e-300)) for t,R in runs.items()}
    rows.append((max(rel.values()), n, rel, g.numel()))
rows.sort()
for m,n,rel,k in rows:
    print(f"{m:9.4f} {k:7d} {n}  " + " ".join(f"{t}={v:.4f}" for t,v in rel.items()))
