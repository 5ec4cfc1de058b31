"""MSheath jump / select pass timing and checksums (A/B of library variants via ASRX_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
from microbench import timeit  # noqa: E402
from asrx import lib  # noqa: E402

dev = torch.device("cuda:0")
tag = os.path.basename(os.environ.get("ASRX_LIB", "prod"))
g = torch.Generator(device=dev).manual_seed(0)
B, L, d = 32, 3001, 384
R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
xin, y, orig, xold = R(B, L, d), R(B, L, d), R(B, L, d), R(B, L, d)
s1, s2 = R(B, L), R(B, L)
alpha, beta, gam = R(B), R(B), R(B, d)
for frac in (1.0, 0.25):
    act = (torch.arange(B, device=dev) < int(B * frac)).float()
    xout = torch.empty_like(xin)
    f1 = lambda: lib.call("asrx_jump_axpy_inplace", lib.ptr(xin), lib.ptr(xout), lib.ptr(s1), lib.ptr(s2), lib.ptr(y),  # noqa: E731
                          lib.ptr(orig), lib.ptr(act), lib.ptr(alpha), lib.ptr(beta), lib.ptr(gam), B, L, d, lib.stream())
    out = torch.empty_like(xin)
    f2 = lambda: lib.call("asrx_jump_select4", lib.ptr(xin), lib.ptr(orig), lib.ptr(xold), lib.ptr(act), lib.ptr(alpha),  # noqa: E731
                          lib.ptr(beta), lib.ptr(gam), lib.ptr(out), B, L, d, lib.stream())
    xip = xin.clone()
    f3 = lambda: lib.call("asrx_jump_axpy_inplace", lib.ptr(xip), lib.ptr(xip), lib.ptr(s1), lib.ptr(s2), lib.ptr(y),  # noqa: E731
                          lib.ptr(orig), lib.ptr(act), lib.ptr(alpha), lib.ptr(beta), lib.ptr(gam), B, L, d, lib.stream())
    t3 = timeit(f3, iters=20)
    t1, t2 = timeit(f1, iters=20), timeit(f2, iters=20)
    torch.cuda.synchronize()
    print(f"{tag} active {frac:4.2f}: jump_axpy_inplace {t1*1e6:7.1f} us (sum {float(xout.double().sum()):.6e})  "
          f"jump_select4 {t2*1e6:7.1f} us (sum {float(out.double().sum()):.6e})  in-place {t3*1e6:7.1f} us", flush=True)
