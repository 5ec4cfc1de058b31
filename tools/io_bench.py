"""Real-data IO path throughput: FLAC decode (native, thread pool) + one pinned
H2D copy + device scaling / peak normalisation (asrx.data.load_batch), on B copies of a 30 s 16 kHz
16-bit mono clip made by the test encoder.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import flac_encode as fe  # noqa: E402
from asrx import data, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
out_dir = os.path.join(ROOT, "gpurun_out", "io_clips")
os.makedirs(out_dir, exist_ok=True)
t0 = time.perf_counter()
w = synth.waveform(1, 30.0)[0].numpy()
pcm = np.round(w * 32767).astype(np.int64)[None]
blob = fe.encode(pcm, 16000, 16, block=4096, plan=lambda f, c: ("lpc", {"order": 8}))
t_enc = time.perf_counter() - t0
paths = []
for i in range(B):
    p = os.path.join(out_dir, f"clip{i}.flac")
    with open(p, "wb") as f:
        f.write(blob)
    paths.append(p)
data.load_batch(paths[:2])  # warm the pool / library
torch.cuda.synchronize()
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    wave, lengths, _ = data.load_batch(paths)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
t = min(ts)
t0 = time.perf_counter()
for p in paths[:4]:
    data.decode_flac(open(p, "rb").read())
t_one = (time.perf_counter() - t0) / 4
print(json.dumps({"clips": B, "flac_bytes_per_clip": len(blob), "compression": round(len(blob) / (2 * pcm.size), 3),
                  "load_batch_s": round(t, 4), "audio_sec_per_sec": round(B * 30.0 / t, 1),
                  "single_clip_decode_ms": round(t_one * 1e3, 2), "threads": data._pool()._max_workers,
                  "encode_s_python": round(t_enc, 1)}))
