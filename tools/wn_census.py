"""Wide-GEMM launches of one probed step grouped by call site (the first frame outside asrx/gemm.py) and shape, with
HIP-event time and the activation operand's storage (ab: bf16 A): where the fp32-A bytes of the step's dominant
kernel come from.  usage: python tools/wn_census.py CONFIG B [TOP]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import prec, probe, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg, B = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
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
_end = probe.end


def end_with_site(kind, e0, work, tag=None):
    site = "?"
    for fr in reversed(traceback.extract_stack()[:-1]):
        if not fr.filename.endswith(("gemm.py", "probe.py")):
            site = f"{os.path.basename(fr.filename)}:{fr.lineno}"
            break
    _end(kind, e0, work, (site,) + tuple(tag or ()))


probe.end = end_with_site
probe.enable(("gemm",))
model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = False
step()
torch.cuda.synchronize()
recs = probe.disable()
by = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
tot = totA32 = 0.0
for w, e0, e1, tag in recs["gemm"]:
    site, kind = tag[0], tag[1]
    if kind not in ("wn", "gact", "router", "lt"):
        continue
    M, N, K = tag[2:5]
    ab = tag[10] if kind == "wn" else (tag[7] if kind == "gact" else (1 if kind == "lt" else 0))
    key = (site, kind, M, N, K, ab) + ((tag[7], tag[11]) if kind == "wn" else ())
    s = e0.elapsed_time(e1) * 1e-3
    by[key][0] += 1
    by[key][1] += s
    by[key][2] += M * K * (2 if ab else 4)
    tot += s
    if not ab:
        totA32 += s
print(f"{cfg} B={B}: wide-GEMM family {tot * 1e3:.2f} ms, of which fp32-A launches {totA32 * 1e3:.2f} ms")
for k, (n, s, ab_bytes, _) in sorted(by.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{str(k):75s} n={n:4d} {s * 1e3:7.2f} ms {s / n * 1e6:8.1f} us  A {ab_bytes / n / 1e6:7.1f} MB/launch")
