"""Host-time diagnosis of the dead-block graph (processor.graph_dead_blocks): per step, the host time of the
forward, of _replay_dead / the eager dead enqueue, of the graph replay call and of the backward; captures counted.
usage: python tools/dead_graph_diag.py CONFIG BATCH STEPS [MODE: graph | eager | eager1 (one side stream)] [steady]
steady: no synchronisation between steps (the bench's timed loop): host times then include blocking on the GPU."""
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

cfg_name, B, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
mode = sys.argv[4] if len(sys.argv) > 4 else "graph"
graph = mode == "graph"
steady = len(sys.argv) > 5 and sys.argv[5] == "steady"
prec.set_precision("bf16")
torch.manual_seed(0)
dev = torch.device("cuda", 0)
model = Model(CONFIGS[cfg_name]).to(dev).train()
P = model.processor
P.graph_dead_blocks = graph
if mode == "eager1":
    one = torch.cuda.Stream()
    P._side_streams = lambda device: (one, one)
wav = synth.waveform(B, 30.0, first_seed=1000).to(dev)
pitch = synth.pitch(B, frames=3001, first_seed=1000, mask_seed=2000).to(dev)
ids, labels = synth.text(B, 256, CONFIGS[cfg_name].tokens, seed=7)
ids, labels = ids.to(dev), labels.to(dev)
T = {}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[name] = T.get(name, 0.0) + time.perf_counter() - t0
    return w


P._replay_dead = timed("replay_dead", P._replay_dead)
model.enc.encode = timed("encode", model.enc.encode)
P._audio = timed("live+dead audio", P._audio)
from asrx import ops as _ops  # noqa: E402
_ops.logits_ce = timed("logits_ce", _ops.logits_ce)
import asrx.model as _am  # noqa: E402
_am.ops.logits_ce = _ops.logits_ce
P._enqueue_dead = timed("enqueue_dead", P._enqueue_dead)
_orig_graph_replay = torch.cuda.CUDAGraph.replay
torch.cuda.CUDAGraph.replay = timed("graph.replay", _orig_graph_replay)
for s in range(steps):
    T.clear()
    if not steady or s == 0:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    spec, wfeat = logmel(wav, layout="BFM", pool=True)
    out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch, waveform=wfeat.unsqueeze(1))
    t1 = time.perf_counter()
    out["loss"].backward()
    t2 = time.perf_counter()
    if not steady:
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"{cfg_name} B={B} {mode} step {s}: fwd host {1e3*(t1-t0):.1f} ms, bwd host {1e3*(t2-t1):.1f} ms, wall {1e3*(t3-t0):.1f} ms, "
          f"graphs {len(P._dgraphs)} seen {len(P._dseen)} | " + ", ".join(f"{k} {1e3*v:.1f} ms" for k, v in T.items()),
          flush=True)
