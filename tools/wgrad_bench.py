"""Weight-gradient GEMM timing at the step's shapes: the register-staged bf16 kernel (asrx_wgrad_bf16)
against the generic split-K LDS-DMA gemm_kernel.  python tools/wgrad_bench.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G, lib, prec  # noqa: E402

dev = torch.device("cuda:0")
prec.set_precision("bf16")
for (R, M, N) in [(192064, 384, 384), (96000, 384, 384), (192064, 384, 1152), (192064, 1536, 384),
                  (192064, 384, 1536), (8192, 384, 384), (8192, 64, 384), (8192, 1152, 384)]:
    dy = torch.randn(R, M, device=dev)
    x = torch.randn(R, N, device=dev)
    out = torch.zeros(M, N, device=dev)
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    sk = G._splitk_for(R, tiles)

    def new():
        lib.call("asrx_wgrad_bf16", lib.ptr(dy), M, lib.ptr(x), N, lib.ptr(out), N, M, N, R, sk, lib.stream())

    def old():
        G.gemm(dy, x, out, M=M, N=N, K=R, lda=M, ldb=N, ldc=N, a_kc=False, b_kc=False, beta=1.0, splitk=sk)

    res = {}
    for name, fn in (("new", new), ("old", old)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / 10
    byts = 4.0 * R * (M + N)
    print(f"R={R} M={M} N={N} sk={sk}: new {res['new']*1e6:.1f} us ({byts/res['new']/1e12:.2f} TB/s, "
          f"{2*R*M*N/res['new']/1e12:.0f} TF/s)  old {res['old']*1e6:.1f} us ({byts/res['old']/1e12:.2f} TB/s)",
          flush=True)
