"""Experimental GEMM variants (not product code): time debug modes of the wide GEMM."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", ".."), os.path.join(HERE, "..", "..", "asr-model_amd")]
import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libexp.so"))
P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


SHAPES = [(192064, 384, 384), (96032, 1536, 384), (96032, 384, 1536)]


def run_p():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    fn = lib.exp_gemm_wnp
    fn.restype = I32
    fn.argtypes = [I32, P, I64, I32, I64, I64, P, I64, P, I64, P, P, I64, I64, I64, F32, F32, I32, I32, P]
    for (M, N, K) in SHAPES:
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        bias = torch.randn(N, device=dev)
        Wb = W.to(torch.bfloat16)
        C = torch.empty(M, N, device=dev)
        ref = (A.to(torch.bfloat16).float() @ Wb.float().t()) + bias
        for nj, nss in ((3, (2, 3)),):
            for ns in nss:
                for cap in ((256,) if nj == 3 else (512,)):
                  for dbg in (0, 8, 16, 24, 6, 14, 30):
                   for swz in (1,):
                    for bb in ((None, bias) if dbg == 0 else (bias,)):
                        f = lambda: fn(swz * 10000000 + dbg * 100000 + ns * 1000 + cap, A.data_ptr(), K, 0, 1, 1, Wb.data_ptr(), K, C.data_ptr(), N,
                                       None if bb is None else bb.data_ptr(), None, M, N, K, 1.0, 0.0, 0, nj, s)
                        C.fill_(float("nan"))
                        rc = f()
                        assert rc == 0, rc
                        torch.cuda.synchronize()
                        r2 = ref if bb is not None else ref - bias
                        if dbg & 7: r2 = C
                        err = float((C - r2).abs().max() / r2.abs().max())
                        t = timeit(f)
                        byts = (M * K + M * N) * 4
                        print(f"wnp M={M} N={N} K={K} nj={nj} ns={ns} cap={cap} dbg={dbg} swz={swz} bias={bb is not None}: {t*1e6:7.1f} us"
                              f"  {byts/t/1e9:6.0f} GB/s {2*M*N*K/t/1e12:6.1f} TF/s err={err:.2e}", flush=True)
        del A, W, Wb, C, ref


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for name in sys.argv[1:] or ["exp_gemm_wn"]:
        fn = getattr(lib, name)
        fn.restype = I32
        fn.argtypes = [I32, P, I64, I32, I64, I64, P, I64, P, I64, P, P, I64, I64, I64, F32, F32, I32, I32, P]
        for (M, N, K) in SHAPES:
            A = torch.randn(M, K, device=dev)
            W = torch.randn(N, K, device=dev)
            Wb = W.to(torch.bfloat16)
            C = torch.empty(M, N, device=dev)
            ref = (A.to(torch.bfloat16).float() @ Wb.float().t())
            for nj in (1, 3):
                for dbg in (0, 1, 2, 4, 3, 7):
                    f = lambda: fn(dbg, A.data_ptr(), K, 0, 1, 1, Wb.data_ptr(), K, C.data_ptr(), N, None, None, M, N,
                                   K, 1.0, 0.0, 0, nj, s)
                    rc = f()
                    assert rc == 0, rc
                    if dbg == 0:
                        torch.cuda.synchronize()
                        err = float((C - ref).abs().max() / ref.abs().max())
                    t = timeit(f)
                    byts = (M * K + M * N) * 4
                    print(f"{name} M={M} N={N} K={K} nj={nj} dbg={dbg}: {t*1e6:7.1f} us  {byts/t/1e9:6.0f} GB/s "
                          f"{2*M*N*K/t/1e12:6.1f} TF/s" + (f"  err={err:.2e}" if dbg == 0 else ""), flush=True)
            del A, W, Wb, C, ref


if __name__ == "__main__":
    if sys.argv[1:] == ["p"]:
        run_p()
    else:
        main()
