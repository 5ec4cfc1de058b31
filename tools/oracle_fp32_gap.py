"""CPU: the oracle restatement run in float32 against itself in float64 (same inputs, keyed noise, the
float64 run's decisions replayed): the intrinsic fp32 error of the reference's own arithmetic on a
case -- the yardstick for the HIP fp32 parity mode.  usage: oracle_fp32_gap.py B seconds T [cfg]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from oracle import model as om  # noqa: E402

B, sec, T = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
cfg = CONFIGS[sys.argv[4] if len(sys.argv) > 4 else "tiny"]
torch.manual_seed(0)
sd = {k: v.detach() for k, v in Model(cfg).state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, 0)
ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}


def run(dtype, dec):
    P = {k: (v.to(dtype).requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
    om.use_decisions(dec)
    try:
        r = om.forward(P, ocfg, x["text_ids"], x["labels"], spectrogram=x["spectrogram"].to(dtype),
                       pitch=x["pitch"].to(dtype), waveform=x["waveform"].to(dtype), seed=7, step=3, training=True,
                       live_only=True, dtype=dtype)
        r["loss"].backward()
    finally:
        om.use_decisions(None)
    return P, r


rec = om.Decisions()
P64, r64 = run(torch.float64, rec)
rp = om.Decisions(table=rec.rec)
P32, r32 = run(torch.float32, rp)
print("replayed", rp.replayed, "overridden", rp.overridden, "cond overridden", rp.cond_overridden)
lg = r32["logits"].detach().double()
lr = r64["logits"].detach()
print(f"fp32 oracle vs fp64 oracle: logits rel {float((lg - lr).abs().max() / lr.abs().max()):.3e}")
gmax = max(float(P64[n].grad.abs().max()) for n in P64 if torch.is_tensor(P64[n]) and P64[n].grad is not None)
rows = []
for n in P64:
    if not torch.is_tensor(P64[n]) or P64[n].grad is None or ".router." in n or ".depth.bias" in n:
        continue
    d = float((P32[n].grad.double() - P64[n].grad).abs().max())
    rows.append((d / gmax, d / max(float(P64[n].grad.abs().max()), 1e-30), n))
rows.sort(reverse=True)
print(f"grads: global max {rows[0][0]:.3e} ({rows[0][2]}), own max {max(r[1] for r in rows):.3e}")
for r in rows[:6]:
    print(f"  global {r[0]:.3e} own {r[1]:.3e} {r[2]}")
