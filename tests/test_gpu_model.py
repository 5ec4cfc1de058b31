"""Whole-model parity: the HIP Model (fp32 parity mode) against the oracle forward (float64 CPU) on
identical parameters, inputs and keyed noise — logits, argmax ids, loss and parameter gradients."""
import pytest
import torch

from oracle import model as om

pytestmark = pytest.mark.gpu


def _toy_inputs(B=2, T=8, S=101, V=1000, seed=1):
    g = torch.Generator().manual_seed(seed)
    spec = torch.randn(B, 128, S, generator=g)
    pitch = torch.rand(B, 1, S, generator=g) * 200
    wav = torch.randn(B, 1, S - 1, generator=g) * 0.1
    ids = torch.randint(3, V, (B, T), generator=g)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1)
    labels[1, -2:] = 0  # some ignored positions
    return spec, pitch, wav, ids, labels


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("train", [True, False])
def test_model_parity_fp32(cuda, train):
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=128, head=2, layer=4, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).cuda()
    model.train(train)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    spec, pitch, wav, ids, labels = _toy_inputs()
    seed, step = 7, 3
    model.set_noise(seed, step)
    with prec.precision("fp32"):
        out = model(labels=labels.cuda(), text_ids=ids.cuda(), spectrogram=spec.cuda(), pitch=pitch.cuda(),
                    waveform=wav.cuda())
        out["loss"].backward()
    P = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
    ref = om.forward(P, {"dims": 128, "head": 2, "layer": 4}, ids, labels, spectrogram=spec, pitch=pitch,
                     waveform=wav, seed=seed, step=step, training=train)
    ref["loss"].backward()
    lg, lr = out["logits"].detach().cpu().double(), ref["logits"].detach()
    err = float(((lg - lr).abs() / lr.abs().max()).max())
    print("logits rel err", err, "loss", float(out["loss"]), float(ref["loss"]))
    assert err < 1e-3
    assert torch.equal(lg.argmax(-1), lr.argmax(-1))
    assert abs(float(out["loss"]) - float(ref["loss"])) / abs(float(ref["loss"])) < 1e-3
    if not train:
        return
    names = dict(model.named_parameters())
    checked = 0
    for name in ["processor.token.weight", "processor.position", "processor.ln.mode_router.0.weight",
                 "processor.block.3.attn.q.1.weight", "processor.block.3.attn.kv.1.weight",
                 "processor.block.3.jump.layers.0.v_gate.mkey", "processor.block.3.mlp.2.weight",
                 "processor.block.3.jump.pnet.net.0.weight", "processor.block.3.jump.jump_s",
                 "enc.conv1.0.weight", "enc.conv2.0.weight", "enc.encoder.0.3.depth.weight",
                 "enc.encoder.1.1.parametrizations.weight.original1", "enc.encoder.0.3.bn.weight"]:
        pg = names[name].grad
        rg = P[name].grad
        assert pg is not None and rg is not None, name
        e = _rel(pg, rg)
        print(name, e)
        assert e < 5e-3, (name, e)
        checked += 1
    assert checked == 14
    # dead blocks get no gradient in either implementation (model.py:617-628)
    assert names["processor.block.0.attn.q.1.weight"].grad is None


def test_skip_dead_blocks_is_output_identical(cuda):
    """processor.skip_dead_blocks (the separately reported bench mode) skips blocks 0..L-2, which the
    reference computes and discards (model.py:617-628): logits, loss and every gradient are
    identical to the faithful run (keyed noise leaves no RNG stream to keep in step).  So are the faithful
    runs with the dead blocks serially on one stream, and with the round-3 schedule (dead audio on the
    main stream, dead text beside it); the default runs whole dead blocks on side streams, joined at the
    end of the backward."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=128, head=2, layer=3, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).cuda().train()
    spec, pitch, wav, ids, labels = _toy_inputs()
    res = []
    # (skip, dead text beside the dead audio, whole dead blocks on side streams across the backward); the
    # default schedule runs three times: its reruns measure the spread the float-atomic parameter-gradient
    # sums give ONE schedule, the yardstick of the schedule gaps
    sched = ((False, True, True), (False, True, True), (False, True, True), (True, True, True),
             (False, False, False), (False, True, False))
    for skip, conc, blocks in sched:
        model.processor.skip_dead_blocks = skip
        model.processor.concurrent_dead_text = conc
        model.processor.concurrent_dead_blocks = blocks
        model.zero_grad(set_to_none=True)
        model.set_noise(3, 1)
        with prec.precision("bf16"):
            out = model(labels=labels.cuda(), text_ids=ids.cuda(), spectrogram=spec.cuda(), pitch=pitch.cuda(),
                        waveform=wav.cuda())
            assert (model.processor._pending is not None) == (blocks and not skip)
            out["loss"].backward()
        assert model.processor._pending is None  # joined at the end of the backward
        res.append((out["logits"].detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters()
                                                     if p.grad is not None}))
    with torch.no_grad(), prec.precision("bf16"):  # no backward to come: joined by the forward itself
        model.processor.concurrent_dead_blocks = True
        model(labels=labels.cuda(), text_ids=ids.cuda(), spectrogram=spec.cuda(), pitch=pitch.cuda(),
              waveform=wav.cuda())
        assert model.processor._pending is None
    model.processor.skip_dead_blocks = False
    model.processor.concurrent_dead_text = True
    # rerun spread of the default schedule, per parameter (the data gradient is deterministic; the parameter
    # gradients' float-atomic sums are not)
    spread = {n: max(_rel(res[i][1][n], res[0][1][n]) for i in (1, 2)) for n in res[0][1]}
    worst_spread = max((v, n) for n, v in spread.items())
    print("rerun spread of one schedule (worst):", worst_spread)
    # a schedule may move a gradient by no more than a small multiple of what a rerun moves it (plus one fp32
    # ulp of headroom at the gradient's scale, for parameters whose three reruns happened to agree bitwise)
    bound = 4.0 * worst_spread[0] + 2.0 ** -23
    # an absolute ceiling beside the relative bound: a regression that made reruns far less reproducible would
    # raise the relative bound with it
    assert worst_spread[0] < 1e-4, worst_spread
    for other in res[1:]:  # reruns, skipped dead blocks, dead blocks serially, the round-3 schedule
        assert torch.equal(res[0][0], other[0])
        assert set(res[0][1]) == set(other[1])
        worst = max((_rel(other[1][n], res[0][1][n]), n) for n in res[0][1])
        print("schedule gap (worst):", worst, "bound", bound)
        assert worst[0] <= min(bound, 1e-4), (worst, worst_spread)


def test_dead_block_graph_matches_eager(cuda):
    """Blocks 0..L-2 replayed from the processor's HIP graph (processor.graph_dead_blocks) run the eager dead
    blocks' kernels: at the capture step's noise the last dead block's output is bit-identical to the eager one,
    and the step's logits equal the eager schedule's (gradients within the float-atomic rerun spread).  The
    first step runs eagerly (the bulk bf16 arena the graph reads is planned during it), the second captures and
    replays, the third replays only."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=128, head=2, layer=3, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).cuda().train()
    proc = model.processor
    proc.keep_dead_out = True
    spec, pitch, wav, ids, labels = _toy_inputs()

    def run(graph):
        proc.graph_dead_blocks = graph
        model.zero_grad(set_to_none=True)
        model.set_noise(3, 1)
        with prec.precision("bf16"):
            out = model(labels=labels.cuda(), text_ids=ids.cuda(), spectrogram=spec.cuda(), pitch=pitch.cuda(),
                        waveform=wav.cuda())
            out["loss"].backward()
        torch.cuda.synchronize()
        return (out["logits"].detach().clone(), {n: p.grad.clone() for n, p in model.named_parameters()
                                                 if p.grad is not None}, proc.dead_out.detach().clone())

    run(False)  # plans the bulk bf16 arena
    ref = run(False)
    assert not proc._dgraphs
    got = [run(True), run(True)]
    assert len(proc._dgraphs) == 1  # captured once, replayed twice
    for g in got:
        assert torch.equal(g[2], ref[2])  # the dead blocks' own result
        assert torch.equal(g[0], ref[0])
        assert set(g[1]) == set(ref[1])
        worst = max((_rel(g[1][n], ref[1][n]), n) for n in ref[1])
        print("graph vs eager gradient gap (worst):", worst)
        assert worst[0] < 1e-4, worst
    proc.reset_dead_graphs()
    assert not proc._dgraphs
    proc.graph_dead_blocks = False


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_forward_is_deterministic(cuda, precision):
    """The forward has no atomics (MSheath's pooled / mem means reduce fixed row chunks in order), so
    two runs of the same step give bit-identical logits: the model's hard decisions (gumbel argmax,
    v_gate thresholds, MSheath jumps) must not depend on float atomic ordering, or parity at the
    benchmarked dims would change from run to run."""
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
    model = Model(cfg).cuda().train()
    spec, pitch, wav, ids, labels = _toy_inputs(B=2, T=16, S=1001)
    outs = []
    for _ in range(2):
        model.set_noise(5, 2)
        with prec.precision(precision):
            out = model(labels=labels.cuda(), text_ids=ids.cuda(), spectrogram=spec.cuda(), pitch=pitch.cuda(),
                        waveform=wav.cuda())
        outs.append((out["logits"].detach().clone(), float(out["loss"])))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
