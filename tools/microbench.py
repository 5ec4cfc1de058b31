"""Ad-hoc kernel timing on the GPU box (not part of the product)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]

import torch  # noqa: E402


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


def gemm_bench():
    from asrx import gemm as G

    dev = torch.device("cuda:0")
    for (M, N, K) in [(192064, 384, 384), (96032, 384, 384), (8192, 384, 384), (96032, 1536, 384), (96032, 384, 1536), (96032, 1152, 384), (96032, 384, 1152), (8192, 40000, 384),
                      (4096, 4096, 4096)]:
        x = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        for p in (1,):
            y = torch.empty(M, N, device=dev)
            t = timeit(lambda: G.gemm(x, W, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, precision=p))
            print(f"gemm prec={p} M={M} N={N} K={K}: {t*1e6:.1f} us  {2*M*N*K/t/1e12:.1f} TF/s", flush=True)
        Wb = G.weight_bf16(W)
        for nj in (1, 2, 3):
            y = torch.empty(M, N, device=dev)
            G._nj_override = nj
            t = timeit(lambda: G.gemm_wn(x, Wb, y, M=M, N=N, K=K, lda=K, ldc=N))
            print(f"  wide nj={nj}: {t*1e6:.1f} us  {2*M*N*K/t/1e12:.1f} TF/s", flush=True)
        G._nj_override = None
        dy = torch.randn(M, N, device=dev)
        t = timeit(lambda: G.linear_wgrad(dy, x))
        print(f"  wgrad bf16: {t*1e6:.1f} us {2*M*N*K/t/1e12:.1f} TF/s", flush=True)
        t = timeit(lambda: G.linear_dgrad(dy, W))
        print(f"  dgrad bf16: {t*1e6:.1f} us {2*M*N*K/t/1e12:.1f} TF/s", flush=True)
        del x, W, y, dy
    ref_a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ref_a @ ref_a)
    print(f"torch bf16 4096^3 (hipBLASLt, reference point): {2*4096**3/t/1e12:.1f} TF/s")


def mel_bench():
    from asrx.mel import logmel

    dev = torch.device("cuda:0")
    B, N = 32, 480000
    wav = torch.randn(B, N, device=dev)
    for lay in ("BFM", "BMF"):
        t = timeit(lambda: logmel(wav, layout=lay, pool=True))
        F = 1 + N // 160
        byts = B * (N * 4 + 128 * F * 4 + (N // 160) * 4)
        print(f"logmel {lay} B={B}: {t*1e6:.1f} us  {byts/t/1e9:.0f} GB/s (algorithmic)", flush=True)


def rowops_bench():
    from asrx import ops

    ops.DIRECT = False  # torch.autograd.grad over parameters below
    dev = torch.device("cuda:0")
    B, T, C = 64, 3001, 384
    x = torch.randn(B, T, C, device=dev)
    g = torch.randn(B, T, C, device=dev)
    nb = B * T * C * 4
    for K in (3, 15):
        w = torch.randn(C, 1, K, device=dev, requires_grad=True)
        b = torch.randn(C, device=dev, requires_grad=True)
        xr = x.clone().requires_grad_(True)
        t = timeit(lambda: ops.DWConv.apply(x, w, b))
        print(f"dwconv fwd K={K}: {t*1e6:.1f} us {2*nb/t/1e9:.0f} GB/s", flush=True)
        y = ops.DWConv.apply(xr, w, b)
        t = timeit(lambda: torch.autograd.grad(y, (xr, w, b), g, retain_graph=True))
        print(f"dwconv bwd K={K}: {t*1e6:.1f} us {3*nb/t/1e9:.0f} GB/s (dx+dw)", flush=True)
    w = torch.rand(C, device=dev, requires_grad=True)
    b = torch.randn(C, device=dev, requires_grad=True)
    xr = x.clone().requires_grad_(True)
    t = timeit(lambda: ops.BatchNormPS.apply(x, w, b, 1e-5, None))
    print(f"bn fwd: {t*1e6:.1f} us {3*nb/t/1e9:.0f} GB/s (stats + apply)", flush=True)
    y = ops.BatchNormPS.apply(xr, w, b, 1e-5, None)
    t = timeit(lambda: torch.autograd.grad(y, (xr, w, b), g, retain_graph=True))
    print(f"bn bwd: {t*1e6:.1f} us {5*nb/t/1e9:.0f} GB/s", flush=True)


def norm_bench():
    from asrx import lib

    dev = torch.device("cuda:0")
    P = lib.ptr
    for rows, d in ((192064, 384), (8192, 384), (48016, 768)):
        x = torch.randn(rows, d, device=dev)
        w, b = torch.randn(d, device=dev), torch.randn(d, device=dev)
        y = torch.empty_like(x)
        mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        t = timeit(lambda: lib.call("asrx_layernorm_fwd", P(x), P(w), P(b), P(y), P(mean), P(rstd), rows, d, 1e-5,
                                    lib.stream()))
        print(f"ln fwd rows={rows} d={d}: {t*1e6:.1f} us {2*rows*d*4/t/1e9:.0f} GB/s", flush=True)
        g = torch.randn_like(x)
        dx = torch.empty_like(x)
        dw, db = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
        t = timeit(lambda: lib.call("asrx_layernorm_bwd", P(g), P(x), P(w), P(mean), P(rstd), P(dx), P(dw), P(db),
                                    rows, d, lib.stream()))
        print(f"ln bwd rows={rows} d={d}: {t*1e6:.1f} us {3*rows*d*4/t/1e9:.0f} GB/s", flush=True)
        out = torch.zeros(d, device=dev)
        t = timeit(lambda: lib.call("asrx_colsum", P(x), P(out), rows, d, lib.stream()))
        print(f"colsum rows={rows} d={d}: {t*1e6:.1f} us {rows*d*4/t/1e9:.0f} GB/s", flush=True)


def abby_bench():
    """AbbyNormal row kernels at the model's shapes; ck = float64 checksums of the outputs (compare two
    builds with ASRX_LIB: the kernels are deterministic except the dW2 atomics)."""
    from asrx import lib

    dev = torch.device("cuda:0")
    P = lib.ptr
    ck = lambda *ts: " ".join(f"{float(t.double().sum()):.9e}" for t in ts)  # noqa: E731
    for rows, d in ((192064, 384), (96032, 384), (1152384, 64), (48016, 768)):
        g0 = torch.Generator(device=dev).manual_seed(rows + d)
        x = torch.randn(rows, d, device=dev, generator=g0) * 3
        lg = torch.randn(rows, 3, device=dev, generator=g0)
        b2 = torch.randn(3, device=dev, generator=g0)
        out = torch.empty_like(x)
        outb = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
        ys = torch.empty(rows, 3, device=dev)
        idx = torch.empty(rows, dtype=torch.int32, device=dev)
        t = timeit(lambda: lib.call("asrx_abby_fwd_logits", P(x), P(lg), P(b2), P(out), P(ys), P(idx), rows, d, 1, 1,
                                    0, 7, 1, lib.stream()))
        print(f"abby fwd rows={rows} d={d}: {t*1e6:.1f} us {2*rows*d*4/t/1e9:.0f} GB/s (x in, out) ck {ck(out, ys)}",
              flush=True)
        t = timeit(lambda: lib.call("asrx_abby_fwd_logits2", P(x), P(lg), P(b2), P(outb), 1, P(ys), P(idx), rows, d,
                                    1, 1, 0, 7, 1, None, None, None, lib.stream()))
        print(f"abby fwd bf16-out rows={rows} d={d}: {t*1e6:.1f} us {rows*d*6/t/1e9:.0f} GB/s ck {ck(outb)}",
              flush=True)
        h = torch.randn(rows, d, device=dev, generator=g0)
        w2 = torch.randn(3, d, device=dev, generator=g0)
        g = torch.randn(rows, d, device=dev, generator=g0)
        dx, dh = torch.empty_like(x), torch.empty_like(x)
        dW2, db2 = torch.zeros(3, d, device=dev), torch.zeros(3, device=dev)
        t = timeit(lambda: lib.call("asrx_abby_bwd", P(g), P(x), P(h), P(w2), P(ys), P(idx), P(dx), P(dh), P(dW2),
                                    P(db2), rows, d, lib.stream()))
        print(f"abby bwd rows={rows} d={d}: {t*1e6:.1f} us {5*rows*d*4/t/1e9:.0f} GB/s (g,x,h in; dx,dh out) "
              f"ck {ck(dx, dh)}", flush=True)
        dx.zero_()
        t = timeit(lambda: lib.call("asrx_abby_bwd2", P(g), P(x), P(h), P(w2), P(ys), P(idx), P(dx), P(dh), P(dW2),
                                    P(db2), rows, d, 1, lib.stream()), iters=1, warm=0)
        print(f"abby bwd acc rows={rows} d={d}: {t*1e6:.1f} us (one launch, cold) ck {ck(dx, dh)}", flush=True)
        del x, h, g, dx, dh, out, outb


def msrow_bench():
    """MSheath layer row passes (asrx_msheath_row_fwd2 / _bwd) at the tiny config's shape (B=32 x 6002 rows, d=384,
    M=64, Dh=192), all samples at the layer and half of them; ck = float64 checksums of the outputs."""
    from asrx import lib

    dev = torch.device("cuda:0")
    P = lib.ptr
    ck = lambda *ts: " ".join(f"{float(t.double().sum()):.9e}" for t in ts)  # noqa: E731
    B, L, d, M, Dh = 32, 6002, 384, 64, 192
    rows, N = B * L, M + Dh
    g0 = torch.Generator(device=dev).manual_seed(5)
    rn = lambda *s: torch.randn(*s, device=dev, generator=g0)  # noqa: E731
    x, SH = rn(rows, d), rn(rows, N)
    lnw, lnb, gw, gb = rn(d), rn(d), rn(d) * 0.05, rn(1)
    mval, w2, b2, cw, cb = rn(M), rn(Dh) * 0.05, rn(1), rn(2), rn(1)
    tx = torch.full((1,), 0.3, device=dev)
    px = torch.empty(rows, d, device=dev)
    sc = [torch.empty(rows, device=dev) for _ in range(7)]
    for frac, tag in ((1.0, "all"), (0.5, "half")):
        next_i = torch.where(torch.arange(B, device=dev) < int(B * frac), 1.0, 2.0).float()
        fwd = lambda: lib.call("asrx_msheath_row_fwd2", P(x), P(lnw), P(lnb), P(gw), P(gb), P(SH), N, P(mval),  # noqa
                               P(w2), P(b2), P(cw), P(cb), P(tx), P(px), 0, *[P(t) for t in sc], rows, d, M, Dh,
                               1e-5, d ** -0.5, P(next_i), 1, L, lib.stream())
        t = timeit(fwd)
        nb = rows * frac * (2 * d + N) * 4
        print(f"msheath row fwd {tag}: {t*1e6:.1f} us {nb/t/1e9:.0f} GB/s ck {ck(px, *sc)}", flush=True)
        dpx, dg, dion = rn(rows, d), rn(rows), rn(rows)
        dx = torch.zeros(rows, d, device=dev)
        grads = [torch.zeros(n, device=dev) for n in (d, d, d, 1, M, Dh, 1, 2, 1, Dh)]
        dSH = torch.empty(rows, N, device=dev)
        bwd = lambda: lib.call("asrx_msheath_row_bwd", P(dpx), P(x), P(lnw), P(lnb), P(sc[0]), P(sc[1]), P(dg),  # noqa
                               P(sc[3]), P(gw), P(dion), P(SH), N, P(sc[2]), P(mval), P(w2), P(cw), P(sc[5]),
                               P(sc[6]), P(dx), P(grads[0]), P(grads[1]), P(grads[2]), P(grads[3]), P(dSH),
                               P(grads[4]), P(grads[5]), P(grads[6]), P(grads[7]), P(grads[8]), P(grads[9]),
                               rows, d, M, Dh, d ** -0.5, P(next_i), 1, L, lib.stream())
        t = timeit(bwd)
        nb = rows * frac * (4 * d + 2 * N) * 4
        dx.zero_()
        bwd()
        print(f"msheath row bwd {tag}: {t*1e6:.1f} us {nb/t/1e9:.0f} GB/s ck {ck(dx, dSH)}", flush=True)


def gact_bench():
    """Linear + act forward and backward in perf mode with the pre-activation stored (asrx_act_bwd_bias) or
    recomputed by the backward's GEMM (asrx_gemm_wn_gact), at the model's MLP shapes."""
    from asrx import gemm as G
    from asrx import ops, prec

    ops.DIRECT = False  # torch.autograd.grad over parameters below
    dev = torch.device("cuda:0")
    for M, N, act in ((192064, 1536, "silu"), (192064, 1152, "gelu"), (96000, 1536, "silu"), (8192, 1536, "silu")):
        x = torch.randn(M, 384, device=dev).to(torch.bfloat16)
        W = (torch.randn(N, 384, device=dev) * 0.05).requires_grad_(True)
        b = (torch.randn(N, device=dev) * 0.1).requires_grad_(True)
        gy = torch.randn(M, N, device=dev)
        for rec in (False, True):
            G.RECOMPUTE_ACT = rec
            with prec.precision("bf16"):
                tf = timeit(lambda: ops.linear(x, W, b, act=act), iters=10)
                y = ops.linear(x, W, b, act=act)
                tb = timeit(lambda: torch.autograd.grad(y, (W, b), gy, retain_graph=True), iters=10)
            print(f"linear+{act} M={M} N={N} recompute={rec}: fwd {tf*1e6:.1f} us  bwd {tb*1e6:.1f} us  "
                  f"total {(tf+tb)*1e6:.1f} us", flush=True)
        G.RECOMPUTE_ACT = True
        del x, W, b, gy, y


def attn_bench():
    from asrx import ops, prec

    dev = torch.device("cuda:0")
    for (B, H, Lq, Lk, causal) in [(64, 6, 3001, 3001, False), (32, 6, 256, 3001, False), (32, 6, 256, 256, True)]:
        q = torch.randn(B, Lq, H, 64, device=dev)
        k = torch.randn(B, Lk, H, 64, device=dev)
        v = torch.randn(B, Lk, H, 64, device=dev)
        fl = 4.0 * B * H * Lq * Lk * 64 * (0.5 if causal else 1.0)
        with prec.precision("bf16"):
            for old in (False, True):
                if old:
                    os.environ["ASRX_ATTN_OLD"] = "1"
                else:
                    os.environ.pop("ASRX_ATTN_OLD", None)
                t = timeit(lambda: ops.attention(q, k, v, causal), iters=5)
                print(f"attn fwd {'old' if old else 'mf '} B={B} H={H} Lq={Lq} Lk={Lk} causal={causal}: "
                      f"{t*1e6:.1f} us {fl/t/1e12:.1f} TF/s", flush=True)
            os.environ.pop("ASRX_ATTN_OLD", None)
            with prec.attention("fp8"):
                t = timeit(lambda: ops.attention(q, k, v, causal), iters=5)
            print(f"attn fwd fp8 B={B} H={H} Lq={Lq} Lk={Lk} causal={causal}: {t*1e6:.1f} us {fl/t/1e12:.1f} TF/s",
                  flush=True)
            for old in (False, True):
                if old:
                    os.environ["ASRX_ATTN_OLD"] = "1"
                else:
                    os.environ.pop("ASRX_ATTN_OLD", None)
                qr, kr, vr = (t_.clone().requires_grad_(True) for t_ in (q, k, v))
                y = ops.attention(qr, kr, vr, causal)
                gy = torch.randn_like(y)
                t = timeit(lambda: torch.autograd.grad(y, (qr, kr, vr), gy, retain_graph=True), iters=3)
                print(f"attn bwd {'old' if old else 'mf '} B={B} Lq={Lq} Lk={Lk}: {t*1e6:.1f} us "
                      f"{2.5*fl/t/1e12:.1f} TF/s", flush=True)
            os.environ.pop("ASRX_ATTN_OLD", None)
        del q, k, v


def attnf_bench():
    """bf16 attention forward only (ASRX_ATTN_VARIANT picks the kernel variant), with its error vs fp32 SDPA."""
    from asrx import ops, prec

    dev = torch.device("cuda:0")
    v = os.environ.get("ASRX_ATTN_VARIANT", "0")
    for (B, H, Lq, Lk, causal) in [(64, 6, 3001, 3001, False), (32, 6, 256, 3001, False)]:
        g = torch.Generator(device=dev).manual_seed(0)
        q, k, vv = (torch.randn(B, L, H, 64, device=dev, generator=g) for L in (Lq, Lk, Lk))
        fl = 4.0 * B * H * Lq * Lk * 64
        with prec.precision("bf16"):
            t = timeit(lambda: ops.attention(q, k, vv, causal), iters=10)
            y = ops.attention(q, k, vv, causal)
        ref = torch.nn.functional.scaled_dot_product_attention(q[:2].transpose(1, 2), k[:2].transpose(1, 2),
                                                               vv[:2].transpose(1, 2)).transpose(1, 2)
        err = float((y[:2] - ref).abs().max() / ref.abs().max())
        print(f"variant {v} attn fwd B={B} H={H} Lq={Lq} Lk={Lk}: {t*1e6:.1f} us {fl/t/1e12:.1f} TF/s "
              f"err {err:.3e} sum {float(y.double().sum()):.6f}", flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["gemm", "mel"]
    if "mel" in what:
        mel_bench()
    if "gemm" in what:
        gemm_bench()
    if "rowops" in what:
        rowops_bench()
    if "attn" in what:
        attn_bench()
    if "attnf" in what:
        attnf_bench()
    if "abby" in what:
        abby_bench()
    if "norm" in what:
        norm_bench()
    if "msrow" in what:
        msrow_bench()
    if "gact" in what:
        gact_bench()
