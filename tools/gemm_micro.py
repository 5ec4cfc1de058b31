"""GPU micro-benchmark of the wide GEMM in isolation (no other stream competing): average kernel time of
back-to-back launches per (M, N, K, A dtype, nj), to separate a shape's own cost from the interference
seen in the step's kernel trace.  usage: python tools/gemm_micro.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402
from asrx import prec  # noqa: E402

prec.set_precision("bf16")
if os.environ.get("GEMM_VARIANT"):  # 1: two-workgroups-per-CU kernel (default), 0: one workgroup per CU
    from asrx import lib  # noqa: E402
    lib.load().asrx_set_gemm_variant(int(os.environ["GEMM_VARIANT"]))
dev = torch.device("cuda:0")
SHAPES = [(8192, 384, 384), (8192, 384, 1536), (8192, 1536, 384), (8192, 1152, 384), (32, 128, 384),
          (192064, 384, 384), (192064, 1536, 384), (192064, 384, 1536)]
# GEMM_SHAPES="M,N,K;M,N,K" / GEMM_NJ="3" / GEMM_ITERS / GEMM_ABF="0,1": a subset (PMC passes)
if os.environ.get("GEMM_SHAPES"):
    SHAPES = [tuple(int(v) for v in t.split(",")) for t in os.environ["GEMM_SHAPES"].split(";")]
NJS = tuple(int(v) for v in os.environ.get("GEMM_NJ", "1,2,3").split(","))
ABFS = tuple(bool(int(v)) for v in os.environ.get("GEMM_ABF", "0,1").split(","))
ITERS = int(os.environ.get("GEMM_ITERS", "50"))
BETA = float(os.environ.get("GEMM_BETA", "0"))  # 1: the accumulating input-gradient launches (C += A W^T)
for M, N, K in SHAPES:
    for abf in ABFS:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16 if abf else torch.float32)
        W = torch.randn(N, K, device=dev) * 0.05
        Wb = G.weight_bf16(W, cache=False)
        C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16 if os.environ.get("GEMM_CBF") else torch.float32)
        bias = torch.randn(N, device=dev) if os.environ.get("GEMM_BIAS") else None
        for nj in NJS:
            if 128 * nj > ((N + 127) // 128) * 128:
                continue
            G._nj_override = nj
            for _ in range(3):
                G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N, bias=bias, beta=BETA)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = ITERS
            e0.record()
            for _ in range(n):
                G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N, bias=bias, beta=BETA)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            print(f"M{M:7d} N{N:5d} K{K:5d} A{'bf16' if abf else 'fp32'} nj{nj}: {us:8.1f} us "
                  f"{2.0 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)
        G._nj_override = 0
