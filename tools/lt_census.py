"""Count the launches of one bench step per GEMM entry point (asrx.lib.CENSUS) and the share of GEMM flops that took
the library path.  usage: python tools/lt_census.py CONFIG BATCH"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import lib, prec, probe, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg, B = sys.argv[1], int(sys.argv[2])
prec.set_precision("bf16")
torch.manual_seed(0)
dev = torch.device("cuda:0")
model = Model(CONFIGS[cfg]).to(dev).train()
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
ids, labels = synth.text(B, 256, CONFIGS[cfg].tokens)
ids, labels = ids.to(dev), labels.to(dev)


def step():
    spec, wf = logmel(wav, layout="BFM", pool=True)
    out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch, waveform=wf.unsqueeze(1))
    out["loss"].backward()
    model.zero_grad(set_to_none=True)


step()
step()
torch.cuda.synchronize()
probe.enable(("gemm",))
model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = False
step()
torch.cuda.synchronize()
recs = probe.disable()
by = collections.defaultdict(lambda: [0, 0.0, 0.0])
for w, e0, e1, tag in recs["gemm"]:
    k = tag[0] if tag else "?"
    by[k][0] += 1
    by[k][1] += w
    by[k][2] += e0.elapsed_time(e1) * 1e-3
tot = sum(v[1] for v in by.values())
for k, (n, w, s) in sorted(by.items(), key=lambda kv: -kv[1][2]):
    print(f"{cfg} B={B} {k:7s} launches {n:6d} flops {w / 1e12:8.3f} TF ({100 * w / tot:5.1f} %) time {s * 1e3:8.2f} ms "
          f"-> {w / max(s, 1e-12) / 1e12:7.1f} TF/s")
