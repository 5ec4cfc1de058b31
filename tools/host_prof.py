"""Host-side (Python) profile of the eager headline step on the GPU box: cProfile over K steps after W warm-ups,
then the top functions by own time and by cumulative time.  The step is near host-bound in eager mode
(bench.py host_issue_ms_per_step), so this is where the host's share of the step goes.
usage: host_prof.py [config] [B] [K]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.dist import GradSync  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
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
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(K):
    step()
pr.disable()
th = time.perf_counter() - t0
torch.cuda.synchronize()
tw = time.perf_counter() - t0
print(f"{K} steps: host issue {th / K * 1e3:.1f} ms/step (under cProfile), wall {tw / K * 1e3:.1f} ms/step")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(60)
