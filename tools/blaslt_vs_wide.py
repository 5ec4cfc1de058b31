"""Library GEMM (torch.nn.functional.linear on bf16 -> hipBLASLt / rocBLAS on ROCm) against the asrx wide GEMM on the
model's plain product shapes (bf16 activations, bf16 weights, bias; asrx with fp32 and bf16 out, the library bf16
out): average time of back-to-back launches.  Decides whether plain GEMMs should go to the library (allowed for plain
library GEMMs).  usage: python tools/blaslt_vs_wide.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from asrx import gemm as G  # noqa: E402
from asrx import prec  # noqa: E402

prec.set_precision("bf16")
dev = torch.device("cuda:0")
SHAPES = [(192064, 384, 384), (192064, 1152, 384), (192064, 384, 1152), (192064, 1536, 384), (192064, 384, 1536),
          (48016, 768, 768), (48016, 2304, 768), (48016, 768, 2304), (48016, 3072, 768), (48016, 768, 3072),
          (48016, 1024, 1024), (48016, 3072, 1024), (48016, 1024, 3072), (8192, 1152, 384), (2048, 2304, 768)]


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


for M, N, K in SHAPES:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    Wb16 = W.to(torch.bfloat16)
    Wb = G.weight_bf16(W, cache=False)
    C = torch.empty(M, N, device=dev)
    Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    ours = t(lambda: G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
    ours_b = t(lambda: G.gemm_wn(A, Wb, Cb, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
    bb = b.to(torch.bfloat16)
    lib_b = t(lambda: F.linear(A, Wb16, bb))  # bf16 out, bias
    print(f"M{M:7d} N{N:5d} K{K:5d}: asrx f32-out {ours:7.1f} us ({fl / ours / 1e6:6.0f} TF/s) bf16-out {ours_b:7.1f} us "
          f"({fl / ours_b / 1e6:6.0f}) | library bf16-out {lib_b:7.1f} us ({fl / lib_b / 1e6:6.0f} TF/s)", flush=True)
