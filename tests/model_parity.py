"""Whole-model parity harness: the HIP Model against the oracle restatement (oracle/model.py, float64
CPU) on identical parameters, synthetic LibriSpeech-shaped inputs and keyed noise.

Test infrastructure (imports oracle/); used by tests/test_gpu_model_configs.py and
tools/parity_probe.py.  The metrics follow SURVEY.md §8(d) "Parity gates":
  logits_max  max |HIP - oracle| / max |oracle|          (the 1e-3 relative gate of north_star)
  logits_rms  rms(HIP - oracle) / rms(oracle)
  argmax      fraction of text positions whose argmax token id agrees
  loss        |loss_HIP - loss_oracle| / |loss_oracle|
  grads       max |g_HIP - g_oracle| / max |g_oracle| for selected parameters
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from oracle import mel as omel
from oracle import model as om

GRAD_PARAMS = ["processor.token.weight", "processor.position", "processor.ln.mode_router.0.weight",
               "processor.block.{L1}.attn.q.1.weight", "processor.block.{L1}.attn.kv.1.weight",
               "processor.block.{L1}.attn.out.1.weight", "processor.block.{L1}.mlp.2.weight",
               "processor.block.{L1}.mlp.4.weight", "processor.block.{L1}.jump.mlp.0.weight",
               "enc.conv1.0.weight", "enc.conv2.0.weight", "enc.encoder.0.3.point1.weight",
               "enc.encoder.{L1}.1.parametrizations.weight.original1"]


def inputs(B: int, seconds: float, T: int, vocab: int, seed: int = 0):
    """Synthetic clips (asrx.synth) -> the reference's feature dict through the float64
    oracle front end: spectrogram (B, 128, S), pitch (B, 1, S), waveform (B, 1, S - 1), text."""
    from asrx import synth

    wav = synth.waveform(B, seconds, first_seed=1000 + seed)
    spec = torch.stack([torch.from_numpy(omel.log_mel(w.numpy().astype(np.float64))).float() for w in wav])
    wf = torch.stack([torch.from_numpy(omel.waveform_feature(w.numpy())).float() for w in wav])  # (B, 1, S-1)
    S = spec.shape[-1]
    pitch = synth.pitch(B, frames=S, first_seed=1000 + seed, mask_seed=2000 + seed)
    ids, labels = synth.text(B, T, vocab, seed=7 + seed)
    return {"spectrogram": spec, "pitch": pitch, "waveform": wf, "text_ids": ids, "labels": labels}


_ORACLE_CACHE: dict = {}


def _rel_max(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def compare(cfg, B=1, seconds=30.0, T=256, precision="bf16", train=True, grads=True, seed=0, noise=(7, 3),
            model_seed=0, device="cuda"):
    """Run the HIP Model and the oracle on the same inputs; return a dict of metrics."""
    from asrx import prec
    from asrx.model import Model

    torch.manual_seed(model_seed)
    model = Model(cfg).to(device)
    model.train(train)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    x = inputs(B, seconds, T, cfg.tokens, seed)
    model.set_noise(*noise)
    t0 = time.perf_counter()
    with prec.precision(precision):
        out = model(labels=x["labels"].to(device), text_ids=x["text_ids"].to(device),
                    spectrogram=x["spectrogram"].to(device), pitch=x["pitch"].to(device),
                    waveform=x["waveform"].to(device))
        if grads:
            out["loss"].backward()
    torch.cuda.synchronize()
    t_gpu = time.perf_counter() - t0
    ck = (repr(cfg), B, seconds, T, train, seed, noise, model_seed)
    t0 = time.perf_counter()
    if ck not in _ORACLE_CACHE:  # the oracle depends on the case only, not on the HIP precision
        P = {k: (v.double().requires_grad_(True) if v.is_floating_point() else v) for k, v in sd.items()}
        ref = om.forward(P, {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}, x["text_ids"], x["labels"],
                         spectrogram=x["spectrogram"], pitch=x["pitch"], waveform=x["waveform"], seed=noise[0],
                         step=noise[1], training=train, live_only=True)
        ref["loss"].backward()
        _ORACLE_CACHE[ck] = (P, {"logits": ref["logits"].detach(), "loss": float(ref["loss"])})
    P, ref = _ORACLE_CACHE[ck]
    t_ref = time.perf_counter() - t0
    lg = out["logits"].detach().double().cpu()
    lr = ref["logits"].detach()
    res = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer, "tokens": cfg.tokens, "B": B, "S": x["pitch"].shape[-1],
           "T": T, "precision": precision, "train": train,
           "logits_max": _rel_max(lg, lr),
           "logits_rms": float((lg - lr).pow(2).mean().sqrt() / lr.pow(2).mean().sqrt()),
           "argmax": float((lg.argmax(-1) == lr.argmax(-1)).double().mean()),
           "loss": abs(float(out["loss"]) - ref["loss"]) / abs(ref["loss"]),
           "loss_hip": float(out["loss"]), "loss_ref": ref["loss"],
           "t_gpu_s": round(t_gpu, 2), "t_oracle_s": round(t_ref, 2)}
    if grads:
        names = dict(model.named_parameters())
        ge = {}
        for n in GRAD_PARAMS:
            n = n.format(L1=cfg.layer - 1)
            pg, rg = names[n].grad, P[n].grad
            ge[n] = None if (pg is None or rg is None) else _rel_max(pg.double().cpu(), rg)
        res["grads"] = ge
        res["grads_max"] = max(v for v in ge.values() if v is not None)
    return res
