"""bf16 activation storage (perf mode, asrx.prec.bf16_storage): an activation whose only consumers are
GEMM / attention operands is written bf16 by its producer.  The consumers round their operands to bf16
anyway, so every product must be BIT-IDENTICAL to the fp32-storage path on the same values -- these
tests check exactly that, kernel by kernel, and for the whole model's forward (logits, loss) with the
storage switched on and off.  Gradients may differ only where a backward reads a bf16-stored tensor
for its own fp32 arithmetic (attention's Delta = rowsum(dO * O) with O stored bf16), so they are
compared with a tolerance."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bfr(t):
    """t rounded to bf16 (RNE) and back to fp32."""
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("nj", [1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(5000, 384, 384), (257, 200, 96), (1000, 1152, 64)])
def test_wide_gemm_bf16_a_and_c(cuda, nj, M, N, K):
    from asrx import gemm as G

    g = torch.Generator().manual_seed(M + N + K + nj)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    Wb = G.weight_bf16(W, cache=False)
    G._nj_override = nj
    try:
        ref = torch.empty(M, N, device=cuda)
        zr = torch.empty(M, N, device=cuda)
        G.gemm_wn(_bfr(x), Wb, ref, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act="gelu", Z=zr)
        xb = x.to(torch.bfloat16)
        y = torch.empty(M, N, device=cuda)
        z = torch.empty(M, N, device=cuda)
        G.gemm_wn(xb, Wb, y, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act="gelu", Z=z)
        yb = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        zb = torch.empty(M, N, device=cuda)
        G.gemm_wn(xb, Wb, yb, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act="gelu", Z=zb)
    finally:
        G._nj_override = None
    assert torch.equal(y, ref) and torch.equal(z, zr)  # bf16 A: bit-identical products
    assert torch.equal(zb, zr)
    assert torch.equal(yb, ref.to(torch.bfloat16))  # bf16 C = the fp32 result rounded once


def test_wide_conv3_bf16_a(cuda):
    """k3 implicit im2col over a bf16-stored activation (C % 8 == 0)."""
    from asrx import gemm as G

    g = torch.Generator().manual_seed(9)
    Bn, T, C, O = 3, 301, 128, 384
    x = torch.randn(Bn, T, C, generator=g).to(cuda)
    Wt = (torch.randn(O, 3 * C, generator=g) / (3 * C) ** 0.5).to(cuda)
    Wb = G.weight_bf16(Wt, cache=False)
    ref = torch.empty(Bn, T, O, device=cuda)
    G.gemm_wn(_bfr(x), Wb, ref, M=Bn * T, N=O, K=3 * C, lda=C, ldc=O, conv=True, conv_F=T, conv_C=C)
    y = torch.empty(Bn, T, O, device=cuda)
    G.gemm_wn(x.to(torch.bfloat16), Wb, y, M=Bn * T, N=O, K=3 * C, lda=C, ldc=O, conv=True, conv_F=T, conv_C=C)
    assert torch.equal(y, ref)


@pytest.mark.parametrize("R,M,N", [(8192, 384, 384), (30000, 384, 1152), (777, 64, 200)])
def test_wgrad_bf16_x(cuda, R, M, N):
    """Weight gradient with X stored bf16: the same products as fp32 X rounded to bf16 (the float-atomic
    split-K order aside)."""
    from asrx import gemm as G, prec

    g = torch.Generator().manual_seed(R + M + N)
    dy = torch.randn(R, M, generator=g).to(cuda)
    x = torch.randn(R, N, generator=g).to(cuda)
    with prec.precision("bf16"):
        ref = G.linear_wgrad(dy, _bfr(x))
        got = G.linear_wgrad(dy, x.to(torch.bfloat16))
    scale = float((_bfr(dy).t().abs() @ _bfr(x).abs()).max())
    assert float((got - ref).abs().max()) / scale < 1e-6


@pytest.mark.parametrize("d,H", [(384, 1), (64, 6), (768, 1)])
def test_abby_bf16_out(cuda, d, H):
    from asrx import ops, prec
    from asrx.model import AbbyNormal

    torch.manual_seed(1)
    mod = AbbyNormal(d).cuda()
    x = (torch.randn(3, 500, H, d) * 3).cuda() if H > 1 else (torch.randn(3, 500, d) * 3).cuda()
    with prec.precision("bf16"), torch.no_grad():
        ref = ops.abby_normal(mod, x, 500, H, 0, 77, True, out_bf16=False)
        got = ops.abby_normal(mod, x, 500, H, 0, 77, True, out_bf16=True)
    assert got.dtype == torch.bfloat16
    assert torch.equal(got, ref.to(torch.bfloat16))


@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("Lq,Lk,causal", [(3001, 3001, False), (256, 3001, False), (256, 256, True)])
def test_attention_bf16_io(cuda, hd, Lq, Lk, causal):
    """q / k / v stored bf16 and o stored bf16: forward bit-identical to fp32 storage of the same
    (bf16-representable) values; backward identical too (Delta reads the same values)."""
    from asrx import ops, prec

    g = torch.Generator().manual_seed(Lq + Lk + hd)
    B, H = 2, 3
    q = _bfr(torch.randn(B, Lq, H, hd, generator=g)).to(cuda)
    k = _bfr(torch.randn(B, Lk, H, hd, generator=g)).to(cuda)
    v = _bfr(torch.randn(B, Lk, H, hd, generator=g)).to(cuda)
    go = torch.randn(B, Lq, H, hd, generator=g).to(cuda)
    res = []
    with prec.precision("bf16"):
        for bf in (False, True):
            args = [t.to(torch.bfloat16) if bf else t.clone() for t in (q, k, v)]
            args = [t.requires_grad_() for t in args]
            o = ops.attention(*args, causal, out_bf16=bf)
            assert o.dtype == (torch.bfloat16 if bf else torch.float32)
            o.backward(go)
            res.append((o.detach().float(), [t.grad.float() for t in args]))
    assert torch.equal(res[1][0], res[0][0].to(torch.bfloat16).float())
    # backward: Delta = rowsum(dO * O) reads the bf16-stored O in the second run
    for a, b in zip(res[0][1], res[1][1]):
        assert float((a - b).abs().max() / b.abs().max()) < 2e-2


def test_model_forward_unchanged_by_bf16_storage(cuda):
    """Whole model, perf mode: logits and loss BIT-IDENTICAL with bf16 activation storage on and off
    (every bf16-stored activation is consumed only by operands that were rounded to bf16 anyway);
    parameter gradients within the attention-Delta difference."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).cuda().train()
    model.fused_ce = False  # the fused logits + CE stores bf16 logits (tests/test_gpu_ce_fused.py)
    g = torch.Generator().manual_seed(4)
    B, T, S = 2, 16, 1001
    spec = torch.randn(B, 128, S, generator=g).cuda()
    pitch = (torch.rand(B, 1, S, generator=g) * 200).cuda()
    wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).cuda()
    ids = torch.randint(3, 1000, (B, T), generator=g)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1).cuda()
    ids = ids.cuda()
    res = []
    for on in (False, True):
        model.zero_grad(set_to_none=True)
        model.set_noise(3, 1)
        with prec.precision("bf16"), prec.storage(on):
            out = model(labels=labels, text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wav)
            out["loss"].backward()
        res.append((out["logits"].detach().clone(), float(out["loss"]),
                    {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]
    assert set(res[0][2]) == set(res[1][2])
    # measured against the model's largest gradient; the analytically-zero gradients (identity router,
    # the depthwise-conv bias ahead of the per-sample BatchNorm: rounding residue only) are skipped
    from model_parity import ANALYTIC_ZERO

    gmax = max(float(g.abs().max()) for g in res[0][2].values())
    errs = {n: float((res[1][2][n] - res[0][2][n]).abs().max()) / gmax for n in res[0][2]
            if not any(z in n for z in ANALYTIC_ZERO)}
    worst = max(errs, key=errs.get)
    print("bf16 storage on/off: worst gradient difference", errs[worst], worst)
    assert errs[worst] < 2e-2, (errs[worst], worst)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_msheath_nograd_inplace_step_is_exact(cuda, precision):
    """MSheath without a backward (dead blocks, eval, decoding) skips x_new and updates x in place
    (asrx_jump_axpy_inplace); its output must equal the saving path's bit for bit, with jumps taken
    (samples skipping layers) and the caller's input left untouched."""
    from asrx import msheath, ops, prec
    from asrx.model import MSheath

    torch.manual_seed(2)
    mod = MSheath(384, 6, 4).cuda()
    with torch.no_grad():
        mod.pnet.net[2].bias.copy_(torch.tensor([0.0, 2.0, 2.0]))  # favour jumps
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(5, 300, 384, generator=g) * 2).cuda()
    x_copy = x.clone()
    gpol = ops.policy_noise(5, 4, 0, 1234, x.device)
    with prec.precision(precision), torch.no_grad():
        y0, _ = msheath.forward(mod, x, gpol, save=False)
        y1, sv = msheath.forward(mod, x, gpol, save=True)
    assert torch.equal(x, x_copy)
    assert torch.equal(y0, y1)
    acts = sv["ws"][1][:, 2].cpu()  # per-layer (alpha, beta, active, next_out, mem_v) x B workspace
    assert bool((acts == 0).any()), acts  # some sample skipped a layer
