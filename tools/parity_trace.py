"""GPU debug aid: where does the HIP fp32 forward leave the float64 oracle?  Runs one parity case
(fp32 parity mode, HIP decisions recorded and replayed in the oracle) with every H == 1 AbbyNormal
output recorded per (site key, sample) on both sides, then prints the relative error of each in the
oracle's execution order.  usage: python tools/parity_trace.py [B seconds T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from asrx import decisions as hdec  # noqa: E402
from asrx import ops, prec  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from oracle import model as om  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
sec = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
T = int(sys.argv[3]) if len(sys.argv) > 3 else 64
cfg = CONFIGS["tiny"]
torch.manual_seed(0)
model = Model(cfg).cuda().train()
sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, 0)

hip = {}
_abby = ops.abby_normal


def abby_rec(mod, xx, L, H, sid_base, key, use_noise=True, out_bf16=False, tgate=None):
    y = _abby(mod, xx, L, H, sid_base, key, use_noise, out_bf16, tgate)
    if H == 1:
        yy = y.detach().float().reshape(-1, L, y.shape[-1]).cpu()
        for s in range(yy.shape[0]):
            hip[(int(key) & 0xFFFFFFFF, sid_base + s)] = yy[s].double()
    return y


ops.abby_normal = abby_rec
model.set_noise(7, 3)
hdec.enable()
with prec.precision("fp32"):
    out = model(labels=x["labels"].cuda(), text_ids=x["text_ids"].cuda(), spectrogram=x["spectrogram"].cuda(),
                pitch=x["pitch"].cuda(), waveform=x["waveform"].cuda())
torch.cuda.synchronize()
table = hdec.disable()
ops.abby_normal = _abby

order, ref = [], {}
_rows = om.abby_rows


def rows_rec(P, pre, xx, noise, site, sids):
    y = _rows(P, pre, xx, noise, site, sids)
    k = int(noise.key(site)) & 0xFFFFFFFF
    for s, sid in enumerate(sids):
        ref[(k, sid)] = y[s].detach()
        order.append((site, sid, k))
    return y


om.abby_rows = rows_rec
P = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
rp = om.Decisions(table=table)
om.use_decisions(rp)
with torch.no_grad():
    r = om.forward(P, {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}, x["text_ids"], x["labels"],
                   spectrogram=x["spectrogram"], pitch=x["pitch"], waveform=x["waveform"], seed=7, step=3,
                   training=True, live_only=True)
om.use_decisions(None)
print("replayed", rp.replayed, "overridden", rp.overridden, "cond overridden", rp.cond_overridden)
lg = out["logits"].detach().double().cpu()
print("logits rel", float((lg - r["logits"]).abs().max() / r["logits"].abs().max()))
seen = set()
for site, sid, k in order:
    if (k, sid) in seen or (k, sid) not in hip:
        continue
    seen.add((k, sid))
    a, b = hip[(k, sid)], ref[(k, sid)]
    if a.shape != b.shape:
        print(f"{site:28s} sid {sid}: shape {tuple(a.shape)} vs {tuple(b.shape)}")
        continue
    e = float((a - b).abs().max() / b.abs().max())
    row = int((a - b).abs().max(dim=-1).values.argmax())
    print(f"{site:28s} sid {sid}: rel {e:.3e}  worst row {row}")
