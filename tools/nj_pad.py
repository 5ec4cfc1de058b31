"""Tile width of the wide GEMM when N is not a multiple of the widest tile: the MSheath SH product's N = M + Dh (448 at
small, 576 at medium) pads to 768 columns at nj = 3 but 512 / 768 at nj = 2.  Back-to-back launch time per nj.
usage: python tools/nj_pad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402
from asrx import prec  # noqa: E402

prec.set_precision("bf16")
dev = torch.device("cuda:0")


def t(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for M, N, K in [(48016, 448, 768), (24000, 448, 768), (2048, 448, 768), (192064, 256, 384), (48016, 576, 1024),
                (24000, 576, 1024), (2048, 576, 1024), (48016, 64, 768), (8192, 40000, 384)]:
    W = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    Wb = G.weight_bf16(W, cache=False)
    C = torch.empty(M, N, device=dev)
    line = f"M{M:7d} N{N:6d} K{K:5d} default nj {G._nj(M, N)}:"
    for ab in (0, 1):
        A = torch.randn(M, K, device=dev)
        if ab:
            A = A.to(torch.bfloat16)
        for nj in (1, 2, 3):
            if 128 * nj > ((N + 127) // 128) * 128:
                continue
            G._nj_override = nj
            try:
                us = t(lambda: G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
            finally:
                G._nj_override = None
            line += f" {'bf16' if ab else 'f32 '}A nj{nj} {us:7.1f} us"
    print(line, flush=True)
