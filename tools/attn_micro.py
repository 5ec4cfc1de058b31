"""GPU micro-benchmark of the bf16 flash attention at the step's shapes (bf16-stored q / k / v / o, as the bench
step stores them): forward, and forward + backward.  usage: python tools/attn_micro.py [repeats, default 2]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import ops, prec  # noqa: E402

dev = torch.device("cuda:0")
if os.environ.get("ATTN_VARIANT"):  # asrx_set_attn_variant: 1 software-pipelined forward (default), 0 round-4
    from asrx import lib  # noqa: E402
    lib.load().asrx_set_attn_variant(int(os.environ["ATTN_VARIANT"]))
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
shapes = [(64, 6, 3001, 3001, False), (32, 6, 3000, 3000, False), (32, 6, 256, 3001, False), (16, 12, 3001, 3001, False)]
for rep in range(reps):
    for (B, H, Lq, Lk, causal) in shapes:
        q, k, vv = (torch.randn(B, L, H, 64, device=dev).to(torch.bfloat16) for L in (Lq, Lk, Lk))
        fl = 4.0 * B * H * Lq * Lk * 64 * (0.5 if causal else 1.0)
        with prec.precision("bf16"):
            with torch.no_grad():
                t = timeit(lambda: ops.attention(q, k, vv, causal, out_bf16=True), iters=5)
            qr, kr, vr = (t_.clone().requires_grad_(True) for t_ in (q, k, vv))
            y = ops.attention(qr, kr, vr, causal, out_bf16=True)
            gy = torch.randn_like(y)
            tb = timeit(lambda: torch.autograd.grad(y, (qr, kr, vr), gy, retain_graph=True), iters=3)
        print(f"rep {rep} B={B} H={H} Lq={Lq} Lk={Lk}: fwd {t*1e6:8.1f} us {fl/t/1e12:6.1f} TF/s "
              f"({fl/t/1e12/2500:.3f} of bf16 peak) | bwd {tb*1e6:8.1f} us {2.5*fl/tb/1e12:6.1f} TF/s "
              f"({2.5*fl/tb/1e12/2500:.3f})", flush=True)
        del q, k, vv, qr, kr, vr, y, gy
