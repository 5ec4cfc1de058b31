"""Decision record / replay in the oracle (oracle.model.Decisions), CPU only: a forward replaying its own
recorded decisions reproduces itself exactly, and a replayed table with flipped entries is obeyed."""
import torch

from oracle import model as om


def _toy():
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    cfg = Dimensions(tokens=300, mels=128, dims=128, head=2, layer=2, act="gelu", n_type="AbbyNormal")
    sd = {k: v.detach() for k, v in Model(cfg).state_dict().items()}
    g = torch.Generator().manual_seed(1)
    B, T, S = 2, 8, 41
    x = dict(spectrogram=torch.randn(B, 128, S, generator=g), pitch=torch.rand(B, 1, S, generator=g) * 200,
             waveform=torch.randn(B, 1, S - 1, generator=g) * 0.1)
    ids = torch.randint(3, 300, (B, T), generator=g)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1)
    return cfg, sd, x, ids, labels


def _run(cfg, sd, x, ids, labels, dec):
    P = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
    om.use_decisions(dec)
    try:
        r = om.forward(P, {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}, ids, labels, seed=3, step=1,
                       training=True, live_only=True, **x)
        r["loss"].backward()
    finally:
        om.use_decisions(None)
    return r, P


def test_replay_own_decisions_is_identity():
    cfg, sd, x, ids, labels = _toy()
    rec = om.Decisions()
    r0, P0 = _run(cfg, sd, x, ids, labels, rec)
    kinds = {k[0] for k in rec.rec}
    assert kinds == {"abby", "cond", "ion", "action"}, kinds
    rep = om.Decisions(table=rec.rec)
    r1, P1 = _run(cfg, sd, x, ids, labels, rep)
    assert rep.replayed > 0 and rep.overridden == 0
    assert torch.equal(r0["logits"], r1["logits"])
    for n in P0:
        if P0[n].grad is not None:
            assert torch.equal(P0[n].grad, P1[n].grad), n


def test_replay_obeys_flipped_modes():
    cfg, sd, x, ids, labels = _toy()
    rec = om.Decisions()
    r0, _ = _run(cfg, sd, x, ids, labels, rec)
    table = dict(rec.rec)
    k = next(k for k in table if k[0] == "abby" and k[1] == om.Noise(3, 1, torch.float64).key("final.ln"))
    table[k] = (table[k] + 1) % 3  # every final-norm mode of that sample changed
    rep = om.Decisions(table=table)
    r1, _ = _run(cfg, sd, x, ids, labels, rep)
    assert rep.overridden == table[k].numel()
    assert torch.equal(rep.rec[k], rec.rec[k])  # the recorder keeps the oracle's own choice
    assert not torch.equal(r0["logits"], r1["logits"])
