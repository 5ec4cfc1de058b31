"""Wide-GEMM timing over the step's main shapes (A/B of library variants via ASRX_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import gemm as G  # noqa: E402

dev = torch.device("cuda:0")
tag = os.path.basename(os.environ.get("ASRX_LIB", "prod"))
for (M, N, K) in [(192064, 384, 384), (192064, 1152, 384), (192064, 384, 1152), (192064, 1536, 384),
                  (192064, 384, 1536), (96032, 384, 384), (8192, 384, 384)]:
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    Wb = G.weight_bf16(W)
    y = torch.empty(M, N, device=dev)
    t = timeit(lambda: G.gemm_wn(x, Wb, y, M=M, N=N, K=K, lda=K, ldc=N))
    ref = x[:4096].to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t()
    err = float((y[:4096] - ref).abs().max() / ref.abs().max())
    byts = 4 * M * K + 4 * M * N + 2 * N * K
    print(f"{tag} M={M} N={N} K={K} nj={G._nj(M, N)}: {t*1e6:7.1f} us {byts/t/1e9:5.0f} GB/s err {err:.1e}", flush=True)
    del x, W, Wb, y
