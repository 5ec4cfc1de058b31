"""Perf-mode fusions against their unfused compositions (bf16 mode, same kernels otherwise):
  * LinearRes: r + x W^T + b with the residual add in the out projection's GEMM epilogue (model.py:578-580)
    == add(r, linear(x)) bit for bit in the forward, same gradients;
  * asrx_act_bwd_bias: act' applied, gz stored bf16, bias gradient summed in the same pass ==
    bf16(act_bwd) bit for bit, bias gradient == colsum of the fp32 act_bwd within 1e-5;
  * the encoder stems written straight into the group buffer (ops.join_group) == torch.cat of separate
    stems, gradients identical."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,fused_expected", [(40000, 384, 384, True), (8192, 384, 384, True),
                                                  (700, 512, 512, True), (30000, 256, 384, False)])
def test_linear_residual_matches_add(cuda, M, N, K, fused_expected):
    from asrx import gemm as G
    from asrx import ops, prec

    assert (G._nj(M, N) in (1, 3)) == fused_expected, G._nj(M, N)  # nj 2 falls back to add(r, linear(x))
    g = torch.Generator().manual_seed(M + N + K)
    r = torch.randn(M, N, generator=g).to(cuda)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) * 0.05).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    gy = torch.randn(M, N, generator=g).to(cuda)
    res = []
    for fused in (True, False):
        rr = r.clone().requires_grad_(True)
        xx = x.clone().requires_grad_(True)
        WW = W.clone().requires_grad_(True)
        bb = b.clone().requires_grad_(True)
        with prec.precision("bf16"):
            y = ops.linear_residual(rr, xx, WW, bb) if fused else ops.add(rr, ops.linear(xx, WW, bb))
            if fused:
                assert ("LinearRes" in type(y.grad_fn).__name__) == fused_expected, type(y.grad_fn).__name__
            y.backward(gy)
        res.append((y.detach(), rr.grad, xx.grad, WW.grad, bb.grad))
    d = (res[0][0] - res[1][0]).abs()
    assert torch.equal(res[0][0], res[1][0]), (float(d.max()), int((d > 0).sum()), d.nonzero()[:4].tolist())
    assert torch.equal(res[0][1], res[1][1])
    for a, c in zip(res[0][2:], res[1][2:]):
        assert float((a - c).abs().max() / c.abs().max()) < 1e-5


@pytest.mark.parametrize("act", ["gelu", "silu", "sigmoid"])
@pytest.mark.parametrize("M,N,K,abf", [(20000, 1536, 384, True), (9001, 1152, 384, False), (7000, 1536, 384, True)])
def test_linear_act_recomputed_preact_matches_stored(cuda, act, M, N, K, abf):
    """Linear + act in perf mode with the pre-activation recomputed by the backward's GEMM (gemm_wn_gact)
    against the stored-pre-activation path (asrx_act_bwd_bias): the forward is the same launch without the
    z store (bit-identical y); the recomputed z equals the stored one bit for bit (same tiles, same MFMA
    order), so dx / dW match within the compilers' contraction differences of act' (<= 1e-5 of max) and the
    bias gradient (column-sum order differs) within 1e-5 of the column sums of |gz|."""
    from asrx import gemm as G
    from asrx import ops, prec

    assert G._nj(M, N) == 3
    acts = G.RECOMPUTE_ACTS
    G.RECOMPUTE_ACTS = ("gelu", "silu", "sigmoid")  # the kernel covers all three (GELU is off by policy)
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(cuda)
    if abf:
        x = x.to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(cuda)
    b = (torch.randn(N, generator=g) * 0.1).to(cuda)
    gy = torch.randn(M, N, generator=g).to(cuda)
    res = []
    try:
        for rec in (True, False):
            G.RECOMPUTE_ACT = rec
            xx = x.clone().requires_grad_(not abf)
            WW = W.clone().requires_grad_(True)
            bb = b.clone().requires_grad_(True)
            with prec.precision("bf16"):
                y = ops.linear(xx, WW, bb, act=act)
                assert y.grad_fn is not None
                y.backward(gy)
            res.append((y.detach(), None if abf else xx.grad, WW.grad, bb.grad))
    finally:
        G.RECOMPUTE_ACT = True
        G.RECOMPUTE_ACTS = acts
    assert torch.equal(res[0][0], res[1][0])
    for a, c in zip(res[0][1:3], res[1][1:3]):
        if a is not None:
            assert float((a - c).abs().max() / c.abs().max()) < 1e-5
    gabs = (gy * 1.2).abs().sum(0)  # |act'| <= 1.13 (gelu), 1.1 (silu), 0.25 (sigmoid)
    assert float(((res[0][3] - res[1][3]).abs() / gabs.clamp_min(1e-30)).max()) < 1e-5


@pytest.mark.parametrize("act", ["gelu", "silu", "sigmoid"])
@pytest.mark.parametrize("rows,N", [(5000, 1536), (333, 1152), (64, 384)])
def test_act_bwd_bias_matches_unfused(cuda, act, rows, N):
    from asrx import lib, ops

    g = torch.Generator().manual_seed(rows + N)
    gy = torch.randn(rows, N, generator=g).to(cuda)
    z = (torch.randn(rows, N, generator=g) * 2).to(cuda)
    gz_ref = torch.empty_like(gy)
    lib.call("asrx_act_bwd", lib.ptr(gy), lib.ptr(z), lib.ptr(gz_ref), gy.numel(), ops.ACT[act], lib.stream())
    db_ref = gz_ref.double().sum(0)
    gz = torch.empty(rows, N, dtype=torch.bfloat16, device=cuda)
    db = torch.zeros(N, device=cuda)
    lib.call("asrx_act_bwd_bias", lib.ptr(gy), lib.ptr(z), lib.ptr(gz), lib.ptr(db), rows, N, ops.ACT[act],
             lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(gz, gz_ref.to(torch.bfloat16))
    assert float((db.double() - db_ref).abs().max() / db_ref.abs().max()) < 1e-5


def test_stem_group_matches_cat(cuda):
    from asrx import ops, prec
    from asrx.config import Dimensions
    from asrx.model import AudioEncoder

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    enc = AudioEncoder(cfg.mels, cfg.dims, cfg.head, cfg.layer, cfg.act, cfg.n_type, norm=False, enc=False).to(cuda)
    g = torch.Generator().manual_seed(1)
    B, T = 2, 501
    pitch = (torch.rand(B, 1, T, generator=g) * 200).to(cuda)
    spec = torch.randn(B, 128, T, generator=g).to(cuda)
    gy = torch.randn(2 * B, T, cfg.dims, generator=g).to(cuda)
    res = []
    for grouped in (True, False):
        enc.zero_grad(set_to_none=True)
        with prec.precision("bf16"):
            if grouped:
                buf = torch.empty(2 * B, T, cfg.dims, device=cuda)
                x = ops.join_group(buf, [enc.stem(pitch, out=buf[:B]), enc.stem(spec, out=buf[B:])])
            else:
                x = torch.cat([enc.stem(pitch), enc.stem(spec)], 0)
            x.backward(gy)
        res.append((x.detach().clone(), {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}))
    assert torch.equal(res[0][0], res[1][0])
    assert set(res[0][1]) == set(res[1][1]) and len(res[0][1]) >= 4
    for n in res[0][1]:
        a, c = res[0][1][n], res[1][1][n]
        assert float((a - c).abs().max() / c.abs().max().clamp_min(1e-30)) < 1e-5, n


@pytest.mark.parametrize("d,rows", [(384, 3001), (512, 700), (768, 200)])
def test_abby_residual_matches_add(cuda, d, rows):
    """residual + AbbyNormal(x) with the add in the AbbyNormal kernel (model.py:583) == add(residual,
    AbbyNormal(x)) bit for bit, same gradients (keyed noise identical)."""
    from asrx import ops, prec
    from asrx.model import AbbyNormal

    torch.manual_seed(0)
    mod = AbbyNormal(d).to(cuda)
    g = torch.Generator().manual_seed(d + rows)
    x = (torch.randn(2, rows // 2, d, generator=g) * 3).to(cuda)
    r = torch.randn(2, rows // 2, d, generator=g).to(cuda)
    gy = torch.randn(2, rows // 2, d, generator=g).to(cuda)
    res = []
    for fused in (True, False):
        mod.zero_grad(set_to_none=True)
        xx, rr = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
        with prec.precision("bf16"):
            if fused:
                y = ops.abby_normal(mod, xx, rows // 2, 1, 0, 1234, True, residual=rr)
            else:
                y = ops.add(rr, ops.abby_normal(mod, xx, rows // 2, 1, 0, 1234, True))
            y.backward(gy)
        res.append((y.detach(), xx.grad, rr.grad, {n: p.grad.clone() for n, p in mod.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][2], res[1][2])
    assert float((res[0][1] - res[1][1]).abs().max() / res[1][1].abs().max()) < 1e-6
    for n in res[0][3]:
        a, c = res[0][3][n], res[1][3][n]
        assert float((a - c).abs().max() / c.abs().max().clamp_min(1e-30)) < 1e-5, n


@pytest.mark.parametrize("a_bf16,b_bf16", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("R,M,N,splitk", [(5000, 384, 384, 4), (777, 200, 136, 1), (8192, 1536, 384, 8)])
def test_wgrad_bias_matches_colsum(cuda, a_bf16, b_bf16, R, M, N, splitk):
    """asrx_wgrad_bias (bias gradient summed from the weight-gradient kernel's dY stages) == the weight
    gradient of asrx_wgrad_bf16* plus asrx_colsum of dY."""
    from asrx import lib

    if a_bf16 and M % 8 or b_bf16 and N % 8:
        pytest.skip("bf16 operands need multiples of 8")
    g = torch.Generator().manual_seed(R + M + N)
    dy = torch.randn(R, M, generator=g).to(cuda)
    x = torch.randn(R, N, generator=g).to(cuda)
    dyb = dy.to(torch.bfloat16) if a_bf16 else dy
    xb = x.to(torch.bfloat16) if b_bf16 else x
    dw = torch.zeros(M, N, device=cuda)
    db = torch.zeros(M, device=cuda)
    lib.call("asrx_wgrad_bias", lib.ptr(dyb), a_bf16, M, lib.ptr(xb), b_bf16, N, lib.ptr(dw), N, lib.ptr(db), M, N, R,
             splitk, lib.stream())
    dw_ref = torch.zeros(M, N, device=cuda)
    if a_bf16:
        lib.call("asrx_wgrad_bf16_ab", lib.ptr(dyb), M, lib.ptr(xb), b_bf16, N, lib.ptr(dw_ref), N, M, N, R, splitk,
                 lib.stream())
    else:
        lib.call("asrx_wgrad_bf16_ex", lib.ptr(dyb), M, lib.ptr(xb), b_bf16, N, lib.ptr(dw_ref), N, M, N, R, splitk,
                 lib.stream())
    db_ref = dyb.float().double().sum(0)
    torch.cuda.synchronize()
    assert float((dw - dw_ref).abs().max() / dw_ref.abs().max()) < 1e-5
    assert float((db.double() - db_ref).abs().max() / db_ref.abs().max()) < 1e-5


def _tiny_step(cuda, model, x, n_runs_cfg):
    """Run the bf16 training step once per entry of n_runs_cfg (FUSED_BIAS_GRAD value) with the same noise;
    returns the parameter gradients of each run."""
    from asrx import gemm as G
    from asrx import prec

    res = []
    for fused in n_runs_cfg:
        G.FUSED_BIAS_GRAD = fused
        try:
            model.zero_grad(set_to_none=True)
            model.set_noise(7, 3)
            with prec.precision("bf16"):
                out = model(labels=x["labels"].to(cuda), text_ids=x["text_ids"].to(cuda),
                            spectrogram=x["spectrogram"].to(cuda), pitch=x["pitch"].to(cuda),
                            waveform=x["waveform"].to(cuda))
                out["loss"].backward()
            torch.cuda.synchronize()
        finally:
            G.FUSED_BIAS_GRAD = True
        res.append({n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None})
    return res


def _tiny_model(cuda):
    from asrx.config import Dimensions
    from asrx.model import Model

    import model_parity as mp

    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    torch.manual_seed(0)
    model = Model(cfg).to(cuda).train()
    return model, mp.inputs(1, 3.0, 32, cfg.tokens, 0)


def _grad_gap(a, b):
    """max |a - b| / max |b| per parameter."""
    return {n: float((a[n] - b[n]).abs().max() / b[n].abs().max().clamp_min(1e-30)) for n in b}


def test_backward_is_reproducible(cuda):
    """A whole bf16 training step run twice gives the same gradients up to the order of the parameter
    gradients' own fp32 atomic sums: no float atomic feeds the data gradient (the MSheath jump backward's
    per-sample sums are ordered partials, msheath.DETERMINISTIC), so nothing is amplified through the
    backward's cancellations.  (With the atomic form, one rerun moved enc.conv1.0.bias by 2e-4 of its
    max and another fused/unfused pair by 3.6e-3.)"""
    model, x = _tiny_model(cuda)
    r0, r1 = _tiny_step(cuda, model, x, (True, True))
    assert set(r0) == set(r1)
    gap = _grad_gap(r1, r0)
    worst = sorted(gap.items(), key=lambda t: -t[1])[:5]
    print("rerun gap (worst 5):", worst)
    assert worst[0][1] < 1e-4, worst


def test_model_bias_grads_fused_match_colsum(cuda):
    """Fused bias gradients (summed inside the weight-gradient kernel) against the column sums of the SAME
    dY, inside one backward (gemm.BIAS_CHECK): within 1e-5 of each column's sum of |dY| (fp32 summation
    order; relative to the sum itself heavy cancellation would make any order look inexact).  Then the whole step with the
    fused and with the separate column-sum pass: every parameter gradient within 1e-4 of its own max (the
    data gradient is bit-reproducible, test_backward_is_reproducible; what is left is fp32 atomic order)."""
    from asrx import gemm as G

    model, x = _tiny_model(cuda)
    G.BIAS_CHECK = []
    try:
        _tiny_step(cuda, model, x, (True,))
        checks = G.BIAS_CHECK
    finally:
        G.BIAS_CHECK = None
    assert len(checks) > 10, len(checks)
    bad = []
    for k, (fused, ref, tol, args) in enumerate(checks):
        # two fp32 summation orders of the same column: within 1e-5 of the column's sum of |dY| (plus the
        # rounding of the += into what the bias gradient already held; gemm.BIAS_CHECK's tol)
        e = (fused - ref).abs() / tol.clamp_min(1e-38)
        c = int(e.argmax())
        if float(e[c]) > 1.0:
            bad.append((k, float(e[c]), c, float(fused[c]), float(ref[c]), float(tol[c]), args))
    assert not bad, bad
    res = _tiny_step(cuda, model, x, (True, False))
    assert set(res[0]) == set(res[1])
    gap = _grad_gap(res[0], res[1])
    worst = sorted(gap.items(), key=lambda t: -t[1])[:5]
    print("fused vs unfused gap (worst 5):", worst)
    assert worst[0][1] < 1e-4, worst
