"""Greedy-decode throughput (BASELINE configs[4] shape: generate on 30 s clips), synthetic clips,
random-init weights: time of Model.generate vs the naive reference loop (full processor forward
per token).  usage: decode_bench.py [config] [batch] [new_tokens] [attention: bf16|fp8]
With fp8 attention (BASELINE configs[4]) it also reports the token agreement with the bf16 path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.mel import logmel  # noqa: E402
from asrx.model import Model  # noqa: E402
from asrx.noise import NoiseCtx  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
NT = int(sys.argv[3]) if len(sys.argv) > 3 else 32
ATT = sys.argv[4] if len(sys.argv) > 4 else "bf16"
dev = torch.device("cuda:0")
prec.set_precision("bf16")
torch.manual_seed(0)
m = Model(CONFIGS[cfg_name]).to(dev)
wav = synth.waveform(B, 30.0).to(dev)
pitch = synth.pitch(B).to(dev)
spec, wf = logmel(wav, layout="BFM", pool=True)
kw = dict(spectrogram=spec.transpose(1, 2), pitch=pitch, waveform=wf.unsqueeze(1))
agree = None
if ATT == "fp8":
    y_bf16 = m.generate(**kw, max_new_tokens=NT)
prec.set_attention(ATT)
m.generate(**kw, max_new_tokens=2)
torch.cuda.synchronize()
t0 = time.perf_counter()
y = m.generate(**kw, max_new_tokens=NT)
torch.cuda.synchronize()
t_gen = time.perf_counter() - t0
prec.set_attention("bf16")
if ATT == "fp8":
    n = min(y.shape[1], y_bf16.shape[1])
    agree = round(float((y[:, :n] == y_bf16[:, :n]).double().mean()), 4)
# naive reference loop for a few tokens (every block, full forward per token)
with torch.no_grad():
    noise = NoiseCtx(m.noise_seed, m.noise_step, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc = m.enc.encode([pitch, spec.transpose(1, 2).contiguous(), wf.unsqueeze(1)], noise, B)
    xa = {"a": enc[0], "b": enc[1], "c": enc[2]}
    yn = torch.ones(B, 1, dtype=torch.long, device=dev)
    nn_ = min(NT, 4)
    for _ in range(nn_):
        logits = m.processor(yn, xa, noise, seq=True)
        yn = torch.cat((yn, logits[:, -1].argmax(-1, keepdim=True)), 1)
    torch.cuda.synchronize()
    t_naive = time.perf_counter() - t0
steps = y.shape[1] - 1
print(json.dumps({"config": cfg_name, "batch": B, "new_tokens": steps, "generate_s": round(t_gen, 3),
                  "tokens_per_s": round(B * steps / t_gen, 1), "audio_sec_per_s": round(B * 30.0 / t_gen, 1),
                  "naive_s_for_%d_tokens" % nn_: round(t_naive, 3),
                  "naive_s_per_token_est": round(t_naive / nn_, 3), "dtype": "bf16", "attention": ATT,
                  **({"token_agreement_vs_bf16": agree} if agree is not None else {}),
                  "data": "synthetic clips, random-init weights"}))
