"""GPU pitch throughput at the bench's shape (B x 30 s clips, the reference's dio + stonemask call)
and its agreement with the float64 oracle on one clip.  python tools/pitch_bench.py [B]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from asrx import pitch, synth  # noqa: E402
from oracle import pitch as P  # noqa: E402  (checker only)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
x = synth.waveform(B, 30.0).cuda()
pitch.reference_pitch(x[:2])  # warm-up (plans, code objects)
torch.cuda.synchronize()
t0 = time.perf_counter()
f = pitch.reference_pitch(x)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
t1 = time.perf_counter()
r = P.reference_pitch(x[0].cpu().numpy())
dt_cpu = time.perf_counter() - t1
g = f[0].cpu().numpy()
both = (g > 0) & (r > 0)
print(json.dumps({"clips": B, "seconds_per_clip": 30.0, "gpu_s": round(dt, 4),
                  "gpu_audio_s_per_s": round(B * 30.0 / dt, 1), "oracle_cpu_s_per_clip": round(dt_cpu, 3),
                  "voicing_agreement": float(((g > 0) == (r > 0)).mean()),
                  "max_rel_diff_voiced": float((np.abs(g[both] - r[both]) / r[both]).max()) if both.any() else 0.0,
                  "frames": int(g.shape[0])}))
