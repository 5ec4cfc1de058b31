"""GPU micro-benchmark of the AbbyNormal router GEMM (asrx_gemm_wn_router) at the step's shapes: d = 64 per-head
rows (router64_kernel, default) vs gemm_wr_kernel's router epilogue (ROUTER_VARIANT=21 -> asrx_set_gemm_variant(5 | 16)),
and d = 384.  usage: python tools/router_micro.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import gemm as G, lib  # noqa: E402

dev = torch.device("cuda:0")
for v in (5, 21, 5, 21):
    lib.load().asrx_set_gemm_variant(v)
    for M, d, keep in [(1152384, 64, False), (1152384, 64, True), (576000, 64, False), (49152, 64, False),
                       (192064, 384, False)]:
        x = torch.randn(M, d, device=dev)
        W1 = torch.randn(d, d, device=dev) / d ** 0.5
        b1 = torch.randn(d, device=dev)
        W2 = torch.randn(3, d, device=dev) / d ** 0.5
        t = timeit(lambda: G.router_fwd(x, W1, b1, W2, keep), iters=20)
        nb = M * d * 4 * (2 if keep else 1) + M * 12
        print(f"variant {v} router M={M} d={d} keep={keep}: {t*1e6:8.1f} us {nb/t/1e9:7.0f} GB/s "
              f"{2*M*d*d/t/1e12:6.1f} TF/s", flush=True)
        del x
lib.load().asrx_set_gemm_variant(5)
