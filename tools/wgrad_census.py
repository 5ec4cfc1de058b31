"""Weight-gradient launches of one probed step by shape and operand storage (asrx.gemm._wgrad: probe tag ("wgrad", M, K,
rows, splitk[, kind]) -- kind 1 bf16 X, 2 bf16 dY, 3 both), with HIP-event time, and the same products on the vendor
library (torch.matmul on bf16 operands -> hipBLASLt) for comparison.  usage: python tools/wgrad_census.py CONFIG B"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import prec, probe, synth  # noqa: E402
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
    if tag and tag[0] in ("wgrad", "gemm"):
        key = tag if tag[0] == "wgrad" else ("gemm",) + tuple(tag[2:5])
        by[key][0] += 1
        by[key][1] += w
        by[key][2] += e0.elapsed_time(e1) * 1e-3
tot = sum(v[2] for v in by.values())
print(f"{cfg} B={B}: weight-gradient / generic GEMM time {tot * 1e3:.2f} ms")


def lib_time(M, K, R):
    a = torch.randn(R, M, device=dev, dtype=torch.bfloat16)
    x = torch.randn(R, K, device=dev, dtype=torch.bfloat16)
    for _ in range(2):
        torch.matmul(a.t(), x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.matmul(a.t(), x)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / 10


for k, (n, w, s) in sorted(by.items(), key=lambda kv: -kv[1][2])[:16]:
    lt = None
    if k[0] == "wgrad":
        lt = lib_time(k[1], k[2], k[3])
    print(f"{str(k):42s} n={n:4d} {s * 1e3 / n * 1e3:8.1f} us/launch {w / max(s, 1e-12) / 1e12:7.1f} TF/s"
          + (f" | library bf16 {lt * 1e6:8.1f} us {2.0 * k[1] * k[2] * k[3] / lt / 1e12:7.1f} TF/s" if lt else ""))
