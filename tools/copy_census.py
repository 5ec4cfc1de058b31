"""Where the headline step's torch-side device copies / fills come from (the rocclr copyBuffer / fillBuffer and
FillFunctor launches of the kernel trace): torch.profiler (CPU activity only) over one eager step after warm-ups,
then the Python call sites of aten::copy_ / clone / contiguous / zero_ / fill_ / zeros, by count.
usage: copy_census.py [config] [B]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from asrx import prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.dist import GradSync  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
prec.set_precision("bf16")
cfg = CONFIGS[cfg_name]
torch.manual_seed(0)
model = Model(cfg).to(dev).train()
gsync = GradSync(model)
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
ids, labels = synth.text(B, 256, cfg.tokens)
ids, labels = ids.to(dev), labels.to(dev)


def step():
    gsync.zero_grad()
    spec, wf = logmel(wav, layout="BFM", pool=True)
    out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch, waveform=wf.unsqueeze(1))
    out["loss"].backward()
    gsync.finish()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
OPS = ("aten::copy_", "aten::clone", "aten::contiguous", "aten::zero_", "aten::fill_", "aten::zeros", "aten::cat",
       "aten::to", "aten::_to_copy")
sites = collections.Counter()
for ev in prof.events():
    if ev.name not in OPS:
        continue
    st = [f for f in (ev.stack or []) if "asrx" in f or "model" in f or "bench" in f]
    sites[(ev.name, st[0] if st else "?", str(ev.input_shapes)[:80])] += 1
for (name, site, shp), n in sites.most_common(60):
    print(f"{n:5d}  {name:18s} {site}  {shp}")
