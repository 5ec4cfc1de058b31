"""Calibration only (not product): hipBLASLt (torch.mm, bf16 in / bf16 out, fp32 accumulate) on the wide-GEMM
shapes of the step, beside asrx's own wide GEMM (gemm_wn, bf16 A) on the same shapes -- what a vendor library
reaches on these K = 384..1536 streaming products.  usage: blas_ref.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402

dev = torch.device("cuda:0")
shapes = [(192064, 384, 384), (192064, 1536, 384), (192064, 384, 1536), (192064, 1152, 384), (96000, 384, 384),
          (8192, 384, 384), (8192, 1536, 384), (8192, 384, 1536)]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for M, N, K in shapes:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    Cf = torch.empty(M, N, device=dev, dtype=torch.float32)
    fl = 2.0 * M * N * K
    t_blas = timeit(lambda: torch.mm(A, W.t(), out=Cb))
    t_blas_f = timeit(lambda: torch.matmul(A, W.t()).float())  # bf16 out + a convert pass (no fp32-out mm for bf16)
    bb = 2 * M * K + 2 * N * K + 2 * M * N
    out = [f"M {M:6d} N {N:5d} K {K:5d}: hipBLASLt bf16->bf16 {t_blas:8.1f} us {fl / t_blas / 1e6:6.1f} TF/s "
           f"{bb / t_blas / 1e3:6.0f} GB/s"]
    for cb, C in ((True, Cb), (False, Cf)):
        t = timeit(lambda: G.gemm_wn(A, W, C, M=M, N=N, K=K, lda=K, ldc=N))
        by = 2 * M * K + 2 * N * K + (2 if cb else 4) * M * N
        out.append(f"asrx bf16->{'bf16' if cb else 'fp32'} {t:8.1f} us {fl / t / 1e6:6.1f} TF/s {by / t / 1e3:6.0f} GB/s")
    print(" | ".join(out), flush=True)
