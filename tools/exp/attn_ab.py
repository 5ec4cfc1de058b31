"""MFMA attention fwd/bwd timing at the step's shapes (A/B of library variants via ASRX_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import ops, prec  # noqa: E402

dev = torch.device("cuda:0")
tag = os.path.basename(os.environ.get("ASRX_LIB", "prod"))
for (B, H, Lq, Lk, causal) in [(64, 6, 3001, 3001, False), (32, 6, 3000, 3000, False), (32, 6, 256, 3001, False),
                               (32, 6, 256, 256, True)]:
    q, k, v = (torch.randn(B, L, H, 64, device=dev) for L in (Lq, Lk, Lk))
    fl = 4.0 * B * H * Lq * Lk * 64 * (0.5 if causal else 1.0)
    with prec.precision("bf16"):
        t = timeit(lambda: ops.attention(q, k, v, causal), iters=5)
        qr, kr, vr = (t_.clone().requires_grad_(True) for t_ in (q, k, v))
        y = ops.attention(qr, kr, vr, causal)
        gy = torch.randn_like(y)
        tb = timeit(lambda: torch.autograd.grad(y, (qr, kr, vr), gy, retain_graph=True), iters=3)
    print(f"{tag} B={B} Lq={Lq} Lk={Lk} causal={causal}: fwd {t*1e6:8.1f} us {fl/t/1e12:6.1f} TF/s | "
          f"bwd {tb*1e6:8.1f} us {2.5*fl/tb/1e12:6.1f} TF/s", flush=True)
    del q, k, v, qr, kr, vr, y, gy
