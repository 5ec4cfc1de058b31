"""fp32-activation wide GEMM against converting the activation to bf16 first (one elementwise pass) and running the
bf16-activation GEMM: where N spans several 384-wide tile columns the fp32 path reads and converts A once per column.
Also checks the two give bit-identical products (A is rounded to bf16 with RNE either way).
usage: python tools/a_convert_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402
from asrx import prec  # noqa: E402

prec.set_precision("bf16")
dev = torch.device("cuda:0")


def t(fn, n=20):
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


for M, N, K in [(48016, 768, 768), (24000, 768, 768), (48016, 1536, 768), (48016, 768, 1536), (48016, 2304, 768),
                (48016, 3072, 768), (192064, 768, 384), (192064, 1152, 384), (192064, 1536, 384), (192064, 384, 384),
                (96000, 768, 384), (48016, 1024, 1024), (48016, 4096, 1024), (2048, 768, 768)]:
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    Wb = G.weight_bf16(W, cache=False)
    C1 = torch.empty(M, N, device=dev)
    C2 = torch.empty(M, N, device=dev)
    G.LIBRARY_GEMM = False
    f32 = t(lambda: G.gemm_wn(A, Wb, C1, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
    conv = t(lambda: A.to(torch.bfloat16))
    Ab = A.to(torch.bfloat16)
    both = t(lambda: G.gemm_wn(A.to(torch.bfloat16), Wb, C2, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
    G.LIBRARY_GEMM = True
    lib = t(lambda: G.gemm_wn(A.to(torch.bfloat16), Wb, C2, M=M, N=N, K=K, lda=K, ldc=N, bias=b))
    G.LIBRARY_GEMM = False
    G.gemm_wn(A, Wb, C1, M=M, N=N, K=K, lda=K, ldc=N, bias=b)
    G.gemm_wn(Ab, Wb, C2, M=M, N=N, K=K, lda=K, ldc=N, bias=b)
    torch.cuda.synchronize()
    same = torch.equal(C1, C2)
    print(f"M{M:7d} N{N:5d} K{K:5d} nj f32 {G._nj(M, N, 0)} bf16 {G._nj(M, N, 1)}: fp32-A {f32:7.1f} us | convert "
          f"{conv:6.1f} + bf16-A = {both:7.1f} us (library where eligible {lib:7.1f}) | bit-identical {same}", flush=True)
