"""GPU micro-benchmark of the bf16 flash-attention forward at the step's shapes (bf16-stored q / k / v / o,
as the bench step stores them), per forward kernel variant (asrx_set_attn_variant: 1 pipelined, 0 not).
usage: python tools/attn_micro.py [variants, default "1,0,1,0"]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import lib, ops, prec  # noqa: E402

dev = torch.device("cuda:0")
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,0,1,0").split(",")]
shapes = [(64, 6, 3001, 3001, False), (32, 6, 3000, 3000, False), (32, 6, 256, 3001, False), (16, 12, 3001, 3001, False)]
for v in variants:
    lib.load().asrx_set_attn_variant(v)
    for (B, H, Lq, Lk, causal) in shapes:
        q, k, vv = (torch.randn(B, L, H, 64, device=dev).to(torch.bfloat16) for L in (Lq, Lk, Lk))
        fl = 4.0 * B * H * Lq * Lk * 64 * (0.5 if causal else 1.0)
        with prec.precision("bf16"), torch.no_grad():
            t = timeit(lambda: ops.attention(q, k, vv, causal, out_bf16=True), iters=5)
        print(f"variant {v} B={B} H={H} Lq={Lq} Lk={Lk}: fwd {t*1e6:8.1f} us {fl/t/1e12:6.1f} TF/s "
              f"({fl/t/1e12/2500:.3f} of bf16 peak)", flush=True)
        del q, k, vv
lib.load().asrx_set_attn_variant(1)
