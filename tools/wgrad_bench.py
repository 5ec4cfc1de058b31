"""Weight-gradient GEMM timing at the step's shapes: the register-staged bf16 kernel (asrx_wgrad_bf16)
against the generic split-K LDS-DMA gemm_kernel, and both operands converted to bf16 first plus the both-bf16 kernel
(asrx_wgrad_bf16_ab; conversion included).  python tools/wgrad_bench.py [tiny|small]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G, lib, prec  # noqa: E402

dev = torch.device("cuda:0")
prec.set_precision("bf16")
SHAPES = {"tiny": [(192064, 384, 384), (96000, 384, 384), (192064, 384, 1152), (192064, 1536, 384),
                   (192064, 384, 1536), (8192, 384, 384), (8192, 64, 384), (8192, 1152, 384)],
          "small": [(48016, 768, 768), (24000, 768, 768), (48016, 1536, 768), (24000, 1536, 768), (48016, 384, 768),
                    (24000, 384, 768), (48016, 768, 3072), (48016, 3072, 768)]}
for (R, M, N) in SHAPES[sys.argv[1] if len(sys.argv) > 1 else "tiny"]:
    dy = torch.randn(R, M, device=dev)
    x = torch.randn(R, N, device=dev)
    out = torch.zeros(M, N, device=dev)
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    sk = G._splitk_for(R, tiles)

    def new():
        lib.call("asrx_wgrad_bf16", lib.ptr(dy), M, lib.ptr(x), N, lib.ptr(out), N, M, N, R, sk, lib.stream())

    def old():
        G.gemm(dy, x, out, M=M, N=N, K=R, lda=M, ldb=N, ldc=N, a_kc=False, b_kc=False, beta=1.0, splitk=sk)

    def conv():
        a = dy.to(torch.bfloat16)
        b = x.to(torch.bfloat16)
        lib.call("asrx_wgrad_bf16_ab", lib.ptr(a), M, lib.ptr(b), 1, N, lib.ptr(out), N, M, N, R, sk, lib.stream())

    res = {}
    for name, fn in (("new", new), ("old", old), ("conv", conv)):
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
          f"{2*R*M*N/res['new']/1e12:.0f} TF/s)  old {res['old']*1e6:.1f} us ({2*R*M*N/res['old']/1e12:.0f} TF/s)  "
          f"bf16-convert+ab {res['conv']*1e6:.1f} us ({2*R*M*N/res['conv']/1e12:.0f} TF/s)",
          flush=True)
