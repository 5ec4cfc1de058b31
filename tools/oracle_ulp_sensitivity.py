"""CPU: how far the float64 oracle's gradients move when every fp32 weight is nudged by about one fp32
ulp (relative 2^-24 uniform noise), decisions replayed -- the gradient's conditioning at fp32 input
precision.  Any fp32 implementation rounds its intermediates at that scale, so a case whose gradients
move by e.g. 1e-2 of max|grad| under this nudge cannot be reproduced closer than that by any of them.
usage: oracle_ulp_sensitivity.py B seconds T [cfg] [samples]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import model_parity as mp  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from oracle import model as om  # noqa: E402

B, sec, T = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
cfg = CONFIGS[sys.argv[4] if len(sys.argv) > 4 else "tiny"]
K = int(sys.argv[5]) if len(sys.argv) > 5 else 2
torch.manual_seed(0)
sd = {k: v.detach() for k, v in Model(cfg).state_dict().items()}
x = mp.inputs(B, sec, T, cfg.tokens, 0)
ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}
rec = om.Decisions()
P0, r0 = mp.oracle_run(sd, ocfg, x, rec, torch.float64)
for s in range(K):
    Pk, rk = mp.oracle_run(mp.ulp_nudge(sd, s), ocfg, x, om.Decisions(table=rec.rec), torch.float64)
    d = mp.grad_distance(Pk, P0)
    print(f"nudge {s}: loss rel {abs(rk['loss'] - r0['loss']) / abs(r0['loss']):.2e}  grads global "
          f"{d[0]:.3e} ({d[1]})  cos {d[2]:.7f}", flush=True)
