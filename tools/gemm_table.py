"""Per-shape GEMM / attention timing of one eager training step (GPU box; not part of the product).
Runs the bench workload once eagerly with the HIP-event probe on and prints one row per GEMM shape:
launches, avg us, TF/s, and the fp32-activation byte rate (A + C read/write, bf16 weights).  Every timed
launch is preceded by a spin kernel (probe precise mode, PRECISE cycles, default 60000), so small kernels
are timed without the host's launch latency; the dead blocks run serially (no concurrent streams).
usage: gemm_table.py [config] [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import prec, probe, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
prec.set_precision("bf16")
cfg = CONFIGS[cfg_name]
torch.manual_seed(0)
model = Model(cfg).to(dev).train()
model.set_noise(seed=0, step=0)
model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = False
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
probe.enable(("gemm", "attn", "logmel"), precise_cycles=int(os.environ.get("PRECISE", "60000")))
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record()
step()
t1.record()
torch.cuda.synchronize()
recs = probe.disable()
total = t0.elapsed_time(t1) * 1e-3
print(f"eager step with spin kernels {total*1e3:.1f} ms (not a step time)")
for kind in ("gemm", "attn", "logmel"):
    tab = {}
    for w, e0, e1, tag in recs[kind]:
        byts = probe.gemm_wr_bytes(tag) if kind == "gemm" else None
        w = probe.gemm_flops(tag, w) if kind == "gemm" else w
        if tag and tag[0] == "wn" and tag[11] >= 0:  # row-list launch: group by the rows it computed
            tag = tag[:11] + (("rows", int(probe.aux(tag[11]).item()) * 128),)
        n, wk, sec, b = tab.get(tag, (0, 0.0, 0.0, 0.0))
        tab[tag] = (n + 1, wk + w, sec + e0.elapsed_time(e1) * 1e-3, None if (byts is None) else (b or 0.0) + byts)
    tsum = sum(v[2] for v in tab.values())
    print(f"== {kind}: {sum(v[0] for v in tab.values())} launches, {tsum*1e3:.1f} ms "
          f"({100*tsum/total:.1f}% of step), {sum(v[1] for v in tab.values())/max(tsum,1e-12)/1e12:.1f} TF/s")
    for tag, (n, w, sec, byts) in sorted(tab.items(), key=lambda kv: -kv[1][2]):
        extra = f" {byts/sec/1e9:7.0f} GB/s {byts/n/1e6:8.1f} MB" if byts is not None else ""
        print(f"{n:5d} x {sec/n*1e6:8.1f} us = {sec*1e3:7.2f} ms  {w/sec/1e12:7.1f} TF/s{extra}  {tag}")
