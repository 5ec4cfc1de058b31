"""Fused tied logits + cross entropy (ops.LogitsCE; model.py:629 logits = x @ token.weight^T, model.py:670
F.cross_entropy(ignore_index=0)) against a float64 restatement on the same bf16 operands.

The fused path stores the logits fp32 (the boundary's dtype, model.py:629 .float()) or, opted in, bf16,
and computes the loss from the GEMM's per-tile (max, sum exp) of the stored logits, so the reference loss
is F.cross_entropy of the HIP's own logits in float64 (1e-5); fp32 logits equal the float64 product of
the bf16 operands within 1e-5, bf16 logits its bf16 rounding within one bf16 ulp; the gradients equal the
float64 gradients of that loss within 1e-2 of their max (dz is stored bf16, as the GEMMs round it
anyway)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).double()


@pytest.mark.parametrize("bf16_logits", [False, True])
@pytest.mark.parametrize("rows,V,D", [(256, 40000, 384), (64, 1000, 384), (300, 40000, 512), (33, 4096, 768)])
def test_logits_ce_fused(cuda, rows, V, D, bf16_logits):
    from asrx import ops, prec

    g = torch.Generator().manual_seed(rows + V + D)
    h = (torch.randn(rows, D, generator=g) * 0.5).to(torch.bfloat16)
    W = torch.randn(V, D, generator=g) * 0.05
    labels = torch.randint(3, V, (rows,), generator=g)
    labels[::7] = 0  # ignore_index rows
    hg = h.to(cuda)
    Wg = W.to(cuda).requires_grad_(True)
    sink = ops.GradSink()
    with prec.precision("bf16"):
        hh = hg.clone().requires_grad_(True)
        logits, loss = ops.LogitsCE.apply(hh, Wg, labels.to(cuda), sink, bf16_logits)
        loss.backward()
    torch.cuda.synchronize()
    assert logits.dtype == (torch.bfloat16 if bf16_logits else torch.float32)
    zb = logits.detach().double().cpu()
    zr = h.double() @ _bf(W).t()
    if bf16_logits:  # bf16 of the float64 product of the bf16 operands, within one bf16 ulp
        ulp = zr.abs().clamp_min(1e-30) * 2.0 ** -7
        assert bool(((zb - zr).abs() <= ulp + 1e-6).all()), float(((zb - zr).abs() / ulp).max())
    else:  # the fp32-accumulated product
        assert float((zb - zr).abs().max() / zr.abs().max()) < 1e-5
    # loss: cross entropy (ignore 0, mean over the rest) of the HIP's own stored logits
    lr = F.cross_entropy(zb, labels, ignore_index=0)
    assert abs(float(loss) - float(lr)) / abs(float(lr)) < 1e-5, (float(loss), float(lr))
    # gradients of that loss w.r.t. the bf16 operands
    zq = zb.clone().requires_grad_(True)
    F.cross_entropy(zq, labels, ignore_index=0).backward()
    dz = zq.grad
    dx_r = dz @ _bf(W)
    dW_r = dz.t() @ h.double()
    dx = sink.buf.double().cpu()
    dW = Wg.grad.double().cpu()
    assert float((dx - dx_r).abs().max() / dx_r.abs().max()) < 1e-2
    assert float((dW - dW_r).abs().max() / dW_r.abs().max()) < 1e-2


def test_logits_ce_bad_label_is_nan(cuda):
    """A label outside [0, V) (the reference's F.cross_entropy raises) gives a NaN loss, never an
    out-of-bounds read."""
    from asrx import ops, prec

    rows, V, D = 16, 1000, 384
    h = torch.randn(rows, D).to(torch.bfloat16).to(cuda)
    W = (torch.randn(V, D) * 0.05).to(cuda)
    for bad in (V, -100):
        labels = torch.randint(1, V, (rows,))
        labels[3] = bad
        for bfl in (False, True):
            with prec.precision("bf16"), torch.no_grad():
                _, loss = ops.LogitsCE.apply(h, W, labels.to(cuda), None, bfl)
            assert torch.isnan(loss).item()
        with torch.no_grad():
            z = torch.randn(rows, V).to(cuda)
            assert torch.isnan(ops.CrossEntropy.apply(z, labels.to(cuda))).item()


def test_all_ignored_labels_give_nan_loss(cuda):
    """Every label ignored: F.cross_entropy's mean over zero rows is NaN (model.py:670), in the fused and
    the fp32 cross entropy alike; the gradient of such a loss is zero (every row ignored)."""
    from asrx import ops, prec

    rows, V, D = 16, 1000, 384
    h = torch.randn(rows, D).to(torch.bfloat16).to(cuda)
    W = (torch.randn(V, D) * 0.05).to(cuda).requires_grad_(True)
    labels = torch.zeros(rows, dtype=torch.long).to(cuda)
    assert torch.isnan(F.cross_entropy(torch.randn(rows, V), labels.cpu(), ignore_index=0))
    for bfl in (False, True):
        with prec.precision("bf16"):
            _, loss = ops.LogitsCE.apply(h, W, labels, None, bfl)
        assert torch.isnan(loss).item()
    z = torch.randn(rows, V).to(cuda).requires_grad_(True)
    loss = ops.CrossEntropy.apply(z, labels)
    assert torch.isnan(loss).item()
    loss.backward(torch.ones((), device=cuda))
    assert float(z.grad.abs().max()) == 0.0


def test_model_returns_fp32_logits_in_bf16_mode(cuda):
    """The drop-in boundary: Model.forward's logits are fp32 in perf mode too (model.py:629 .float()),
    with labels (the fused cross entropy) and without; bf16 logits only when opted in."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).to(cuda).train()
    g = torch.Generator().manual_seed(5)
    B, T, S = 1, 8, 101
    spec = torch.randn(B, 128, S, generator=g).to(cuda)
    ids = torch.randint(3, 1000, (B, T), generator=g).to(cuda)
    labels = torch.randint(3, 1000, (B, T), generator=g).to(cuda)
    with prec.precision("bf16"), torch.no_grad():
        assert model(labels=labels, text_ids=ids, spectrogram=spec)["logits"].dtype == torch.float32
        assert model(text_ids=ids, spectrogram=spec)["logits"].dtype == torch.float32
        model.bf16_logits = True
        try:
            assert model(labels=labels, text_ids=ids, spectrogram=spec)["logits"].dtype == torch.bfloat16
        finally:
            model.bf16_logits = False


def test_model_fused_ce_matches_unfused(cuda):
    """Whole model, perf mode: the fused path's loss equals the unfused path's loss computed from the
    same bf16-rounded logits (the forward up to the final norm is shared), and the embedding gradient
    agrees within bf16 rounding."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).to(cuda).train()
    g = torch.Generator().manual_seed(4)
    B, T, S = 2, 16, 301
    spec = torch.randn(B, 128, S, generator=g).to(cuda)
    pitch = (torch.rand(B, 1, S, generator=g) * 200).to(cuda)
    wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).to(cuda)
    ids = torch.randint(3, 1000, (B, T), generator=g)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1).to(cuda)
    ids = ids.to(cuda)
    res = []
    for fused in (True, False):
        model.fused_ce = fused
        model.zero_grad(set_to_none=True)
        model.set_noise(3, 1)
        with prec.precision("bf16"):
            out = model(labels=labels, text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wav)
            out["loss"].backward()
        res.append((out["logits"].detach().float(), float(out["loss"]), model.processor.token.weight.grad.clone()))
    model.fused_ce = True
    assert res[0][0].dtype == torch.float32
    # fused fp32 logits are the unfused GEMM's logits (same tiles, same accumulation order)
    assert torch.equal(res[0][0], res[1][0])
    lr = float(F.cross_entropy(res[0][0].double().cpu().view(-1, 1000), labels.cpu().view(-1), ignore_index=0))
    assert abs(res[0][1] - lr) / lr < 1e-5
    assert abs(res[0][1] - res[1][1]) / res[1][1] < 1e-5
    gdiff = float((res[0][2] - res[1][2]).abs().max() / res[1][2].abs().max())
    assert gdiff < 3e-2, gdiff
