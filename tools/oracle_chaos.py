"""CPU probe: how far do the float64 oracle's parameter gradients move under an fp32-rounding-sized
input perturbation when every RECORDED hard decision (AbbyNormal mode, v_gate threshold, MSheath
action) is replayed?  Differences left come from discrete choices the recorder does not capture.

usage: python tools/oracle_chaos.py [seconds] [T] [eps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from oracle import model as om  # noqa: E402

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
eps = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-7
torch.manual_seed(0)
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg = CONFIGS["tiny"]
model = Model(cfg)
sd = {k: v.detach() for k, v in model.state_dict().items()}
x = mp.inputs(1, sec, T, cfg.tokens, 0)
ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}


def run(dec, pert):
    P = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
    om.use_decisions(dec)
    g = torch.Generator().manual_seed(11)
    spec = x["spectrogram"].double()
    if pert:
        spec = spec * (1 + eps * torch.randn(spec.shape, generator=g, dtype=torch.float64))
    try:
        r = om.forward(P, ocfg, x["text_ids"], x["labels"], spectrogram=spec, pitch=x["pitch"],
                       waveform=x["waveform"], seed=7, step=3, training=True, live_only=True)
        r["loss"].backward()
    finally:
        om.use_decisions(None)
    return P, r


rec = om.Decisions()
P0, r0 = run(rec, False)
rp = om.Decisions(table=rec.rec)
P1, r1 = run(rp, True)
print("replayed", rp.replayed, "overridden", rp.overridden)
gmax = max(float(P0[n].grad.abs().max()) for n in P0 if torch.is_tensor(P0[n]) and P0[n].grad is not None)
rows = []
for n in P0:
    if not torch.is_tensor(P0[n]) or P0[n].grad is None or P1[n].grad is None:
        continue
    a, b = P1[n].grad, P0[n].grad
    own = float(b.abs().max())
    d = float((a - b).abs().max())
    rows.append((d / max(own, 1e-300), d / gmax, own / gmax, n))
rows.sort(reverse=True)
print(f"logits rel {float((r1['logits'] - r0['logits']).abs().max() / r0['logits'].abs().max()):.3e}")
for r in rows[:25]:
    print(f"{r[0]:.3e} own  {r[1]:.3e} global  scale {r[2]:.2e}  {r[3]}")
