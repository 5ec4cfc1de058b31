"""Wide-GEMM ablation timing (ASRX_WN_DBG bits, see csrc/gemm_wn.hip Params::dbg)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import gemm as G  # noqa: E402

dev = torch.device("cuda:0")
for (M, N, K) in [(192064, 384, 384), (192064, 384, 1536)]:
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    Wb = G.weight_bf16(W)
    y = torch.empty(M, N, device=dev)
    t = timeit(lambda: G.gemm_wn(x, Wb, y, M=M, N=N, K=K, lda=K, ldc=N))
    byts = 4 * M * K + 4 * M * N
    print(f"dbg={os.environ.get('ASRX_WN_DBG', '0')} M={M} N={N} K={K}: {t*1e6:.1f} us {byts/t/1e9:.0f} GB/s", flush=True)
