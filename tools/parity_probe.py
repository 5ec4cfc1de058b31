"""Whole-model parity probe: HIP Model vs the oracle at the BASELINE configs' dims, printing one JSON
line of metrics per case (tests/model_parity.py).  Used to calibrate the tolerances stated in
tests/test_gpu_model_configs.py and DESIGN.md §5.

python tools/parity_probe.py [case ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from asrx.config import CONFIGS, Dimensions  # noqa: E402
import model_parity as mp  # noqa: E402

CASES = {
    # name: (config, B, seconds, T)
    "tiny_full": ("tiny", 1, 30.0, 256),
    "tiny_b2": ("tiny", 2, 10.0, 64),
    "small": ("small", 1, 3.0, 32),
    "medium": ("medium", 1, 2.0, 32),
    "refmain": ("reference_main", 2, 5.0, 64),
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)
    torch.set_num_threads(min(16, os.cpu_count() or 8))
    for name in names:
        cfgname, B, sec, T = CASES[name]
        for precision in ("fp32", "bf16"):
            r = mp.compare(CONFIGS[cfgname], B=B, seconds=sec, T=T, precision=precision)
            r["case"] = name
            print(json.dumps(r), flush=True)
