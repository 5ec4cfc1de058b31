"""GPU debug aid: per-parameter gradient agreement (cosine, relative norm) of the HIP fp32 path against
the float64 oracle on one case with the HIP decisions replayed.  usage: grad_debug.py B seconds T [seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from asrx import decisions as hdec  # noqa: E402
from asrx import prec  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from oracle import model as om  # noqa: E402

B, sec, T = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
cfg = CONFIGS["tiny"]
torch.manual_seed(0)
model = Model(cfg).cuda().train()
model.processor.concurrent_dead_text = os.environ.get("CONC", "1") == "1"
model.processor.skip_dead_blocks = os.environ.get("SKIP", "0") == "1"
print("concurrent_dead_text", model.processor.concurrent_dead_text, "skip_dead_blocks", model.processor.skip_dead_blocks)
sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, seed)
model.set_noise(7, 3)
hdec.enable()
with prec.precision("fp32"):
    out = model(labels=x["labels"].cuda(), text_ids=x["text_ids"].cuda(), spectrogram=x["spectrogram"].cuda(),
                pitch=x["pitch"].cuda(), waveform=x["waveform"].cuda())
    out["loss"].backward()
torch.cuda.synchronize()
table = hdec.disable()
P = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
rp = om.Decisions(table=table)
om.use_decisions(rp)
r = om.forward(P, {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}, x["text_ids"], x["labels"],
               spectrogram=x["spectrogram"], pitch=x["pitch"], waveform=x["waveform"], seed=7, step=3,
               training=True, live_only=True)
r["loss"].backward()
om.use_decisions(None)
print("replayed", rp.replayed, "overridden", rp.overridden, "cond", rp.cond_overridden,
      "loss", float(out["loss"]), float(r["loss"]))
rows = []
for n, p in model.named_parameters():
    if p.grad is None or n not in P or P[n].grad is None:
        continue
    a, b = p.grad.double().cpu().reshape(-1), P[n].grad.reshape(-1)
    cos = float(a @ b / (a.norm() * b.norm()).clamp_min(1e-300))
    rows.append((float(b.norm()), cos, float(a.norm() / b.norm().clamp_min(1e-300)), n))
rows.sort(reverse=True)
for nb, cos, rn, n in rows[:int(os.environ.get("TOP", "30"))]:
    print(f"|g| {nb:.3e}  cos {cos:+.4f}  |hip|/|ref| {rn:.4f}  {n}")
