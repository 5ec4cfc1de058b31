"""GPU: whole-model parity metrics per case with the oracle replaying the HIP decisions (record on
for the cases that report agreement).  One JSON line per (case, precision) -> stdout.
usage: python tools/parity_measure.py [case ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import model_parity as mp  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402

CASES = {
    "tiny_full": ("tiny", 1, 30.0, 256, None),
    "tiny_full_refpitch": ("tiny", 1, 30.0, 256, 6001),
    "tiny_b2": ("tiny", 2, 5.0, 64, None),
    "small": ("small", 1, 3.0, 32, None),
    "medium": ("medium", 1, 2.0, 32, None),
    "refmain": ("reference_main", 2, 5.0, 64, None),
}
names = sys.argv[1:] or list(CASES)
for name in names:
    cfg, B, sec, T, pf = CASES[name]
    for precision in ("fp32", "bf16"):
        r = mp.compare(CONFIGS[cfg], B=B, seconds=sec, T=T, precision=precision, grads=True, pitch_frames=pf,
                       decisions=True, replay=True, yardstick=precision == "fp32",
                       sensitivity=2 if precision == "fp32" else 0)
        r.pop("grads", None)
        print(json.dumps({"case": name, **r}), flush=True)
r = mp.compare(CONFIGS["tiny"], B=1, seconds=10.0, T=64, precision="fp32", grads=True, replay=True, hip_mel=True,
               yardstick=True)
r.pop("grads", None)
print(json.dumps({"case": "hip_mel_e2e", **r}), flush=True)
