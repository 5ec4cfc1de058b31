"""GPU: census of the C-ABI launches of one eager training step of the bench workload, by entry point and
calling file:line (count per step and the summed size proxy, see asrx.lib.CENSUS) -- to find which call
sites produce e.g. the remaining elementwise passes.  usage: python tools/call_census.py [cfg] [B] [filter]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import lib, prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
flt = sys.argv[3] if len(sys.argv) > 3 else ""
dev = torch.device("cuda:0")
prec.set_precision("bf16")
cfg = CONFIGS[cfg_name]
torch.manual_seed(0)
model = Model(cfg).to(dev).train()
model.set_noise(seed=0, step=0)
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
ids, labels = synth.text(B, 256, cfg.tokens)
ids, labels = ids.to(dev), labels.to(dev)


def step():
    for p in model.parameters():
        p.grad = None
    spec, wf = logmel(wav, layout="BFM", pool=True)
    out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch, waveform=wf.unsqueeze(1))
    out["loss"].backward()


step()
torch.cuda.synchronize()
lib.CENSUS = collections.Counter()
step()
torch.cuda.synchronize()
c, lib.CENSUS = lib.CENSUS, None
rows = sorted(((c[k], c[k[:2] + ("size",)], k[0], k[1]) for k in c if k[2] == "n" and flt in k[0]), reverse=True)
print(f"{sum(r[0] for r in rows)} launches")
for n, size, name, site in rows[:60]:
    print(f"{n:6d}  size {size / max(n, 1):14.0f}  {name:32s} {site}")
