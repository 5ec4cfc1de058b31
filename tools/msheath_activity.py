"""How many (sample, layer) pairs of the MSheath calls are active in one training step of the bench
workload (diagnostic, GPU box): the masked per-sample trajectories compute every layer for every
sample; this measures the share an active-only schedule would skip.  python tools/msheath_activity.py"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import msheath, prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

prec.set_precision("bf16")
dev = torch.device("cuda:0")
cfg = CONFIGS["tiny"]
B = 32
torch.manual_seed(0)
model = Model(cfg).to(dev).train()
model.set_noise(seed=0, step=0)
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
ids, labels = synth.text(B, 256, cfg.tokens)
stats = collections.defaultdict(lambda: [0, 0, 0])  # rows-weighted: active rows, total rows, calls
orig = msheath.forward


def rec(mod, x0, gpol, save):
    y, sv = orig(mod, x0, gpol, save)
    return y, sv


def patched(mod, x0, gpol, save):
    B_, L, D = x0.shape
    # rerun the control with saving to read `active` (diagnostic only)
    y, sv = orig(mod, x0, gpol, True)
    acts = [float(l["active"].sum()) for l in sv["layers"]]
    key = "audio" if L > 1000 else "text"
    s = stats[key]
    s[0] += sum(acts) * L
    s[1] += len(acts) * B_ * L
    s[2] += 1
    return (y, sv) if save else (y, None)


msheath.forward = patched
spec, wfeat = logmel(wav, layout="BFM", pool=True)
out = model(labels=labels.to(dev), text_ids=ids.to(dev), spectrogram=spec.transpose(1, 2), pitch=pitch,
            waveform=wfeat.unsqueeze(1))
torch.cuda.synchronize()
print(json.dumps({k: {"active_row_share": v[0] / max(v[1], 1), "calls": v[2]} for k, v in stats.items()}))
