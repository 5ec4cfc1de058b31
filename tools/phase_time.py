"""Per-phase GPU time of one eager training step at the bench workload (tiny, B=32 x 30 s, bf16):
HIP events around log-mel, encoder forward, each processor block's forward (audio side / text side),
logits + CE, and the backward.  Dead-block text concurrency off so phases do not overlap."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import model as M, ops, prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "tiny"]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
prec.set_precision("bf16")
torch.manual_seed(0)
model = M.Model(cfg).to(dev).train()
model.processor.concurrent_dead_text = False
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
ids, labels = synth.text(B, 256, cfg.tokens)
ids, labels = ids.to(dev), labels.to(dev)
marks = []


def mark(name):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    marks.append((name, e))


# wrap the pieces of the step
enc_encode = model.enc.encode


def encode(*a, **k):
    mark("encoder_fwd")
    return enc_encode(*a, **k)


model.enc.encode = encode
for i, blk in enumerate(model.processor.block):
    call0, xa0 = blk.call, blk.xa_side

    def call(*a, _c=call0, _i=i, **k):
        mark(f"b{_i}.{'audio' if a[0].shape[0] > B else 'text'}.call")
        return _c(*a, **k)

    def xa(*a, _x=xa0, _i=i, **k):
        mark(f"b{_i}.{'audio' if a[0].shape[0] > B or a[0].shape[1] > 1000 else 'text'}.xa")
        return _x(*a, **k)

    blk.call, blk.xa_side = call, xa
ln_run = model.processor.ln.run


def final_ln(*a, **k):
    mark("logits+ce")
    return ln_run(*a, **k)


model.processor.ln.run = final_ln


def step():
    mark("logmel")
    spec, wfeat = logmel(wav, layout="BFM", pool=True)
    out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch,
                waveform=wfeat.unsqueeze(1))
    mark("backward")
    out["loss"].backward()
    mark("end")


for _ in range(2):
    marks.clear()
    model.zero_grad(set_to_none=True)
    step()
torch.cuda.synchronize()
agg = {}
for (n, e), (_, e2) in zip(marks, marks[1:]):
    key = n.split(".", 1)[1] if n.startswith("b") and not n.startswith("backward") else n
    if n.startswith("b") and not n.startswith("backward"):
        blk = int(n[1:].split(".")[0])
        key = ("dead " if blk < cfg.layer - 1 else "live ") + key
    agg[key] = agg.get(key, 0.0) + e.elapsed_time(e2)
tot = sum(agg.values())
print(json.dumps({"total_ms": round(tot, 2), "phases_ms": {k: round(v, 2) for k, v in sorted(agg.items(), key=lambda x: -x[1])}}))
