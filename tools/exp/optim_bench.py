"""Time the fused MaxFactor step on the tiny model's parameters (tools/exp, not product)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402
from asrx.optim import MaxFactor, reference_param_groups  # noqa: E402

dev = torch.device("cuda:0")
m = Model(CONFIGS["tiny"]).to(dev)
for p in m.parameters():
    p.grad = torch.randn_like(p)
opt = MaxFactor(reference_param_groups(m), lr=2.5e-3, decay=1e-2)
opt.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    opt.step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host {1e3*(t1-t0)/5:.2f} ms/step, wall {1e3*(t2-t0)/5:.2f} ms/step, params {sum(p.numel() for p in m.parameters())}")
