"""Would split-K help the text side's small-M wide GEMMs?  Times M x N x K against the same N with 3x the rows and a
third of K (the work and workgroup count a 3-way split would give, reduction excluded) and M x N x K/3.
usage: python tools/splitk_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402
from asrx import prec  # noqa: E402

prec.set_precision("bf16")
dev = torch.device("cuda:0")
G.LIBRARY_GEMM = False


def t(fn, n=50):
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


def run(M, N, K, ab):
    A = torch.randn(M, K, device=dev)
    if ab:
        A = A.to(torch.bfloat16)
    Wb = G.weight_bf16(torch.randn(N, K, device=dev) * 0.05, cache=False)
    C = torch.empty(M, N, device=dev)
    return t(lambda: G.gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=K, ldc=N))


for (M, N, K) in [(2048, 768, 768), (2048, 448, 768), (2048, 2304, 768), (2048, 768, 3072), (8192, 384, 384),
                  (2048, 1024, 1024)]:
    for ab in (0, 1):
        for s in (2, 3, 4):
            if K % (s * 32):
                continue
            base = run(M, N, K, ab)
            print(f"{'bf16' if ab else 'fp32'} A  {M}x{N}x{K}: {base:6.1f} us | {s * M}x{N}x{K // s}: "
                  f"{run(s * M, N, K // s, ab):6.1f} us | {M}x{N}x{K // s}: {run(M, N, K // s, ab):6.1f} us", flush=True)
