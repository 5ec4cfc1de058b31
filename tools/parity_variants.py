"""Whole-model fp32 parity of tiny_full under implementation variants (diagnostic, GPU box):
which fused path moves the HIP result away from the oracle.  python tools/parity_variants.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from asrx import model as M, ops  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
import model_parity as mp  # noqa: E402

torch.set_num_threads(min(16, os.cpu_count() or 8))
case = sys.argv[1] if len(sys.argv) > 1 else "tiny_full"
CASES = {"tiny_full": ("tiny", 1, 30.0, 256), "tiny_b2": ("tiny", 2, 10.0, 64)}
cfg, B, sec, T = CASES[case]
fork0 = ops.fork
for name in ("default", "composed_msheath", "no_fork", "composed_no_fork"):
    M.MSheath.fused = "composed" not in name
    ops.fork = (lambda x: x) if "no_fork" in name else fork0
    r = mp.compare(CONFIGS[cfg], B=B, seconds=sec, T=T, precision="fp32")
    g = r.pop("grads")
    r["variant"] = name
    r["top_grads"] = dict(sorted(g.items(), key=lambda kv: -(kv[1] or 0))[:5])
    print(json.dumps(r), flush=True)
