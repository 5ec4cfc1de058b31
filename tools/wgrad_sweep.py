"""Weight-gradient GEMM sweep on the GPU box (split-K factor x shape); not part of the product.
usage: ASRX_GEMM_STAGES=2|3 python tools/wgrad_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from microbench import timeit  # noqa: E402


def main():
    from asrx import gemm as G

    dev = torch.device("cuda:0")
    print("stages", os.environ.get("ASRX_GEMM_STAGES", "2"))
    for (R, N, K) in [(192064, 384, 384), (96000, 384, 384), (192064, 384, 1152), (192064, 1536, 384), (8192, 384, 384)]:
        dy = torch.randn(R, N, device=dev)
        x = torch.randn(R, K, device=dev)
        out = torch.zeros(N, K, device=dev)
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        base = G._splitk_for(R, tiles)
        for sk in sorted({max(1, base // 2), base, base * 2, base * 4, base * 8}):
            if R // sk < 64:
                continue
            t = timeit(lambda: G.gemm(dy, x, out, M=N, N=K, K=R, lda=N, ldb=K, ldc=K, a_kc=False, b_kc=False,
                                      beta=1.0, splitk=sk))
            gb = 4 * R * (N + K) / t / 1e9
            print(f"R={R} N={N} K={K} splitk={sk}{'*' if sk == base else ''}: {t*1e6:.1f} us "
                  f"{2*R*N*K/t/1e12:.1f} TF/s {gb:.0f} GB/s", flush=True)
        del dy, x, out


if __name__ == "__main__":
    main()
