"""Whole-model parity harness: the HIP Model against the oracle restatement (oracle/model.py, float64
CPU) on identical parameters, synthetic LibriSpeech-shaped inputs and keyed noise.

Test infrastructure (imports oracle/); used by tests/test_gpu_model_configs.py and
tools/parity_probe.py.  The metrics follow SURVEY.md §8(d) "Parity gates":
  logits_max  max |HIP - oracle| / max |oracle|          (the 1e-3 relative gate of north_star)
  logits_rms  rms(HIP - oracle) / rms(oracle)
  argmax      fraction of text positions whose argmax token id agrees
  loss        |loss_HIP - loss_oracle| / |loss_oracle|
  grads       max |g_HIP - g_oracle| / max |g_oracle| for selected parameters
  decisions   agreement rates of the hard decisions (AbbyNormal modes, v_gate thresholds, MSheath
              actions) between the HIP path and the oracle on the same inputs (asrx/decisions.py)
  replay      the oracle re-run CONSUMING the HIP path's decisions (oracle.model.Decisions): with the
              discrete trajectory shared, every parameter gradient is compared (grads_all_max) --
              differences left are rounding, not decision flips
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


def inputs(B: int, seconds: float, T: int, vocab: int, seed: int = 0, pitch_frames=None):
    """Synthetic clips (asrx.synth) -> the reference's feature dict through the float64
    oracle front end: spectrogram (B, 128, S), pitch (B, 1, S or pitch_frames), waveform (B, 1, S - 1),
    text.  pitch_frames = 2 S - 1 is the reference's own pitch stream (pw.dio(x, sr, frame_period) binds
    frame_period to f0_floor and keeps dio's 5 ms default frames, essentials.py:451-455: 6001 frames for
    a 30 s clip)."""
    from asrx import synth

    wav = synth.waveform(B, seconds, first_seed=1000 + seed)
    spec = torch.stack([torch.from_numpy(omel.log_mel(w.numpy().astype(np.float64))).float() for w in wav])
    wf = torch.stack([torch.from_numpy(omel.waveform_feature(w.numpy())).float() for w in wav])  # (B, 1, S-1)
    S = spec.shape[-1]
    pitch = synth.pitch(B, frames=S if pitch_frames is None else pitch_frames, first_seed=1000 + seed,
                        mask_seed=2000 + seed)
    ids, labels = synth.text(B, T, vocab, seed=7 + seed)
    return {"spectrogram": spec, "pitch": pitch, "waveform": wf, "text_ids": ids, "labels": labels}


_ORACLE_CACHE: dict = {}


def record(case: str, precision: str, res: dict, path=None) -> None:
    """Append one parity case's measured metrics (every scalar / small entry of compare()'s result, the per-
    parameter gradient table left out) as a JSON line to $ASRX_PARITY_LOG (the GPU suite's collector, e.g.
    profiles/r06_parity_metrics.jsonl); a no-op when the variable is unset."""
    import json
    import os

    path = path or os.environ.get("ASRX_PARITY_LOG")
    if not path:
        return

    def clean(v):
        if isinstance(v, dict):
            return {str(k): clean(x) for k, x in v.items()}
        if isinstance(v, (list, tuple)):
            return [clean(x) for x in v][:64]
        if isinstance(v, (np.floating, np.integer)):
            return v.item()
        if isinstance(v, torch.Tensor):
            return v.item() if v.numel() == 1 else None
        return v if isinstance(v, (int, float, str, bool)) or v is None else str(v)

    line = {"case": case, "precision": precision, "time": time.strftime("%Y-%m-%dT%H:%M:%S"),
            **{k: clean(v) for k, v in res.items() if k != "grads"}}
    with open(path, "a") as f:
        f.write(json.dumps(line) + "\n")


def _rel_max(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def agreement(hip: dict, ref: dict) -> dict:
    """Agreement of two decision tables on their common keys: per kind, the fraction of equal entries
    (AbbyNormal modes and v_gate thresholds per position, MSheath actions per (sample, layer))."""
    out = {}
    # mode 2's per-feature max-vs-avg choice, on the rows both sides put in mode 2
    eq = tot = 0
    for k in hip:
        if k[0] != "cond" or k not in ref or ("abby",) + k[1:] not in ref:
            continue
        both = (hip[("abby",) + k[1:]] == 1) & (ref[("abby",) + k[1:]] == 1)  # (L, H)
        a, b = hip[k][both], ref[k][both]
        eq += int((a == b).sum())
        tot += a.numel()
    out["cond"] = (eq / tot) if tot else None
    out["cond_n"] = tot
    for kind in ("abby", "ion", "action"):
        keys = [k for k in hip if k[0] == kind and k in ref]
        eq = tot = 0
        for k in keys:
            a, b = hip[k], ref[k]
            if kind == "action":
                eq += int(a[0] == b[0])
                tot += 1
            else:
                a, b = a.reshape(-1).double(), b.reshape(-1).double()
                eq += int((a == b).sum())
                tot += a.numel()
        out[kind] = (eq / tot) if tot else None
        out[kind + "_n"] = tot
    return out


def _hip_mel_inputs(x, B, seconds, seed, device):
    """The benchmarked front end: the HIP log-mel and waveform pool of the same synthetic clips (the
    oracle keeps its own float64 mel)."""
    from asrx import synth
    from asrx.mel import logmel

    wav = synth.waveform(B, seconds, first_seed=1000 + seed).to(device)
    spec, wf = logmel(wav, layout="BMF", pool=True)
    y = dict(x)
    y["hip_spectrogram"], y["hip_waveform"] = spec, wf.unsqueeze(1)
    return y


# Parameters whose gradient is analytically zero in the reference, so a relative error is meaningless:
#  * residual.router (model.py:545-557): router(x, x, x) = sum_k w_k x with sum_k w_k = 1 is the
#    identity, its weights get no gradient (the HIP path applies it as the identity);
#  * ConvLite's depthwise-conv bias (model.py:113-114): a per-channel constant removed by the
#    per-sample BatchNorm that follows.
ANALYTIC_ZERO = (".router.", ".depth.bias")


def oracle_run(sd, ocfg, x, dec, dtype=torch.float64, noise=(7, 3), train=True):
    """The oracle forward + backward on state dict sd (fresh leaf copies in dtype) with decision
    table dec; returns (params with .grad, {"logits", "loss"})."""
    # a copy even when sd already holds dtype (requires_grad_ on sd's own tensors would leak into later runs)
    P = {k: (v.detach().to(dtype, copy=True).requires_grad_(True) if v.is_floating_point() else v)
         for k, v in sd.items()}
    om.use_decisions(dec)
    try:
        r = om.forward(P, ocfg, x["text_ids"], x["labels"], spectrogram=x["spectrogram"].to(dtype),
                       pitch=x["pitch"].to(dtype), waveform=x["waveform"].to(dtype), seed=noise[0],
                       step=noise[1], training=train, live_only=True, dtype=dtype)
        r["loss"].backward()
    finally:
        om.use_decisions(None)
    return P, {"logits": r["logits"].detach().double(), "loss": float(r["loss"].detach())}


def ulp_nudge(sd, seed):
    """sd with every floating weight scaled by (1 + u 2^-24), u uniform in [-1, 1): inputs an fp32
    implementation cannot tell apart from sd."""
    g = torch.Generator().manual_seed(1000 + seed)
    return {k: (v.detach().double() * (1 + (torch.rand(v.shape, generator=g, dtype=torch.float64) * 2 - 1) * 2.0 ** -24)
                if v.is_floating_point() else v) for k, v in sd.items()}


def grad_distance(Pa, Pb):
    """(max over parameters of max|ga - gb| / the largest |gb| of the model, that parameter, cosine of
    the concatenated gradients); analytically-zero gradients skipped."""
    names = [n for n in Pb if torch.is_tensor(Pb[n]) and Pb[n].grad is not None and Pa[n].grad is not None
             and not any(z in n for z in ANALYTIC_ZERO)]
    gscale = max(float(Pb[n].grad.abs().max()) for n in names)
    worst, wname = 0.0, None
    for n in names:
        d = float((Pa[n].grad.double() - Pb[n].grad.double()).abs().max()) / gscale
        if d > worst:
            worst, wname = d, n
    a = torch.cat([Pa[n].grad.double().reshape(-1) for n in names])
    b = torch.cat([Pb[n].grad.double().reshape(-1) for n in names])
    return worst, wname, float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-300))


def bf16_nudge(sd, seed):
    """sd with every floating weight scaled by (1 + u 2^-9), u uniform in [-1, 1): a perturbation at bf16
    resolution (bf16 keeps 8 mantissa bits)."""
    g = torch.Generator().manual_seed(2000 + seed)
    return {k: (v.detach().double() * (1 + (torch.rand(v.shape, generator=g, dtype=torch.float64) * 2 - 1) * 2.0 ** -9)
                if v.is_floating_point() else v) for k, v in sd.items()}


BF16_POINTS = ("lin", "qkproj", "qk", "pv", "logits")
BF16_STABLE_REL = 0.1  # a parameter's gradient is stable at bf16 resolution if every perturbation moves it <= 10 %


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-300))


def compare(cfg, B=1, seconds=30.0, T=256, precision="bf16", train=True, grads=True, seed=0, noise=(7, 3),
            model_seed=0, device="cuda", decisions=False, replay=False, hip_mel=False, pitch_frames=None,
            yardstick=False, sensitivity=0, bf16_stability=False):
    """Run the HIP Model and the oracle on the same inputs; return a dict of metrics.
    decisions: record both sides' hard decisions and report their agreement.  replay: re-run the oracle
    consuming the HIP decisions and compare every parameter gradient.  hip_mel: feed the HIP model the
    HIP log-mel of the clips (the benchmarked chain), the oracle its float64 mel.  yardstick (with
    replay): also run the oracle in float32 on the same replayed trajectory -- the reference's own
    arithmetic at fp32 -- and report its distance from the float64 oracle (yard_*): the model's fp32
    conditioning, against which the HIP fp32 path is gated.  sensitivity=K (with replay): K float64
    oracle runs on weights nudged by one fp32 ulp (ulp_nudge), the largest gradient move reported as
    ulp_grads_global -- the gradient's conditioning at fp32 input precision.  bf16_stability (with replay and grads): the gradient's
    conditioning at bf16 resolution -- three more float64 oracle runs on the replayed trajectory, one with
    every GEMM / attention operand rounded to bf16 in the forward and the arriving gradients rounded in the
    backward (oracle EMU) and two on weights nudged at bf16 scale (bf16_nudge); per parameter the largest
    relative L2 move of its gradient over the three (bf16_rel: (HIP's distance, that move)).  A parameter
    moved by at most BF16_STABLE_REL is STABLE at bf16 resolution: the HIP bf16 gradient is gated on
    those (bf16_stable_*)."""
    from asrx import decisions as hdec
    from asrx import prec
    from asrx.model import Model

    torch.manual_seed(model_seed)
    model = Model(cfg).to(device)
    model.train(train)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    x = inputs(B, seconds, T, cfg.tokens, seed, pitch_frames)
    if hip_mel:
        x = _hip_mel_inputs(x, B, seconds, seed, device)
    model.set_noise(*noise)
    if decisions or replay:
        hdec.enable()
    t0 = time.perf_counter()
    try:
        with prec.precision(precision):
            out = model(labels=x["labels"].to(device), text_ids=x["text_ids"].to(device),
                        spectrogram=(x["hip_spectrogram"] if hip_mel else x["spectrogram"]).to(device),
                        pitch=x["pitch"].to(device),
                        waveform=(x["hip_waveform"] if hip_mel else x["waveform"]).to(device))
            if grads:
                out["loss"].backward()
        torch.cuda.synchronize()
    finally:
        hip_dec = hdec.disable() if (decisions or replay) else None
    t_gpu = time.perf_counter() - t0
    ocfg = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}

    def run_oracle(dec, dtype=torch.float64):
        return oracle_run(sd, ocfg, x, dec, dtype, noise, train)

    ck = (repr(cfg), B, seconds, T, train, seed, noise, model_seed, pitch_frames)
    t0 = time.perf_counter()
    ref_dec = None
    if decisions:
        rec = om.Decisions()
        P, ref = run_oracle(rec)
        ref_dec = rec.rec
    elif replay:
        P = ref = None
    else:
        if ck not in _ORACLE_CACHE:  # the oracle depends on the case only, not on the HIP precision
            _ORACLE_CACHE[ck] = run_oracle(None)
        P, ref = _ORACLE_CACHE[ck]
    t_ref = time.perf_counter() - t0
    res_extra = {}
    if decisions:
        res_extra["decisions"] = agreement(hip_dec, ref_dec)
    P32 = ref32 = None
    if replay:
        rp = om.Decisions(table=hip_dec)
        P_r, ref_r = run_oracle(rp)
        if yardstick:
            P32, ref32 = run_oracle(om.Decisions(table=hip_dec), torch.float32)
        if sensitivity:
            moves = [grad_distance(oracle_run(ulp_nudge(sd, k), ocfg, x, om.Decisions(table=hip_dec),
                                              torch.float64, noise, train)[0], P_r)
                     for k in range(sensitivity)]
            res_extra["ulp_grads_global"] = max(m[0] for m in moves)
            res_extra["ulp_grads_worst"] = max(moves)[1]
        res_extra["replayed"] = rp.replayed
        res_extra["overridden"] = rp.overridden
        res_extra["cond_overridden"] = rp.cond_overridden
        if P is None:
            P, ref = P_r, ref_r
        else:
            res_extra["replay_logits_max"] = _rel_max(out["logits"].detach().double().cpu(), ref_r["logits"])
            res_extra["replay_loss"] = abs(float(out["loss"]) - ref_r["loss"]) / abs(ref_r["loss"])
            P, ref = P_r, ref_r
    lg = out["logits"].detach().double().cpu()
    lr = ref["logits"].detach()
    res = {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer, "tokens": cfg.tokens, "B": B, "S": x["pitch"].shape[-1],
           "T": T, "precision": precision, "train": train,
           "logits_max": _rel_max(lg, lr),
           "logits_rms": float((lg - lr).pow(2).mean().sqrt() / lr.pow(2).mean().sqrt()),
           "argmax": float((lg.argmax(-1) == lr.argmax(-1)).double().mean()),
           "loss": abs(float(out["loss"]) - ref["loss"]) / abs(ref["loss"]),
           "loss_hip": float(out["loss"]), "loss_ref": ref["loss"],
           "t_gpu_s": round(t_gpu, 2), "t_oracle_s": round(t_ref, 2), **res_extra}
    if grads and replay:  # every parameter that receives a gradient on both sides
        names = dict(model.named_parameters())
        worst, wname, gworst, gwname = 0.0, None, 0.0, None
        missing, residue, per = [], {}, {}
        gscale = max(float(P[n].grad.abs().max()) for n in names if n in P and P[n].grad is not None)
        for n, p in names.items():
            pg, rg = p.grad, P[n].grad if n in P else None
            if any(z in n for z in ANALYTIC_ZERO):
                # analytically zero gradient: both sides may only hold rounding residue (the HIP
                # identity router none at all), measured against the model's largest gradient
                r = max(float(t.abs().max()) if t is not None else 0.0 for t in (pg, rg)) / gscale
                residue[n] = r
                continue
            if (pg is None) != (rg is None or float(rg.abs().max()) == 0.0):
                if pg is None or float(pg.abs().max()) != 0.0:
                    missing.append(n)
                continue
            if pg is None:
                continue
            d = float((pg.double().cpu() - rg).abs().max())
            e = d / max(float(rg.abs().max()), 1e-30)
            per[n] = (e, d / gscale, float(rg.abs().max()) / gscale)
            if e > worst:
                worst, wname = e, n
            if d / gscale > gworst:
                gworst, gwname = d / gscale, n
        # own: max|dg| / max|g_ref| of that parameter; global: max|dg| / the largest gradient of the model
        res["grads_all_max"] = worst
        res["grads_all_worst"] = wname
        res["grads_all_global"] = gworst
        res["grads_all_global_worst"] = gwname
        res["grads_all_top"] = sorted(((round(v[0], 6), round(v[1], 9), round(v[2], 6), k) for k, v in per.items()),
                                      reverse=True)[:8]
        res["grads_missing"] = missing
        res["zero_grad_residue"] = max(residue.values(), default=0.0)
        if bf16_stability:
            # three bf16-resolution perturbations of the float64 oracle on the replayed trajectory: every GEMM /
            # attention operand rounded to bf16 in the forward and the arriving gradients in the backward
            # (oracle EMU), and two weight nudges at 2^-9
            om.EMU.update(BF16_POINTS + ("bwd",))
            try:
                pert = [run_oracle(om.Decisions(table=hip_dec))[0]]
            finally:
                om.EMU.clear()
            pert += [oracle_run(bf16_nudge(sd, k), ocfg, x, om.Decisions(table=hip_dec), torch.float64, noise, train)[0]
                     for k in range(2)]
            rel = lambda a, b: float((a.double().reshape(-1) - b.double().reshape(-1)).norm()  # noqa: E731
                                     / b.double().reshape(-1).norm().clamp_min(1e-300))
            table, stable = {}, []
            for n in per:
                if float(P[n].grad.abs().max()) == 0.0:
                    continue  # no gradient this step (e.g. an MSheath layer every sample jumped over)
                pr = max(rel(Q[n].grad, P[n].grad) for Q in pert)
                table[n] = (rel(names[n].grad.cpu(), P[n].grad), pr)
                if pr <= BF16_STABLE_REL:
                    stable.append(n)
            cat = lambda G, ns: torch.cat([G(n).double().reshape(-1) for n in ns])  # noqa: E731
            every = list(table)
            res["bf16_pert_rel_whole"] = max(rel(cat(lambda n: Q[n].grad, every), cat(lambda n: P[n].grad, every))
                                             for Q in pert)
            res["bf16_hip_rel_whole"] = rel(cat(lambda n: names[n].grad.cpu(), every), cat(lambda n: P[n].grad, every))
            res["bf16_stable"] = stable
            res["bf16_unstable_n"] = len(table) - len(stable)
            res["bf16_rel"] = {n: (round(a, 5), round(b, 5)) for n, (a, b) in table.items()}  # (HIP, perturbations)
            if stable:
                res["bf16_stable_worst"] = max((table[n][0] / max(3 * table[n][1], 0.05), n) for n in stable)
                res["bf16_stable_set"] = (rel(cat(lambda n: names[n].grad.cpu(), stable), cat(lambda n: P[n].grad, stable)),
                                          max(rel(cat(lambda n: Q[n].grad, stable), cat(lambda n: P[n].grad, stable))
                                              for Q in pert))
        # one number over the whole model: cosine of the concatenated gradients
        kept = [n for n in per]
        a = torch.cat([names[n].grad.double().cpu().reshape(-1) for n in kept])
        b = torch.cat([P[n].grad.reshape(-1) for n in kept])
        res["grads_cos"] = float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-300))
        if P32 is not None:
            yg, yo = 0.0, 0.0
            for n in kept:
                d = float((P32[n].grad.double() - P[n].grad).abs().max())
                yg = max(yg, d / gscale)
                yo = max(yo, d / max(float(P[n].grad.abs().max()), 1e-30))
            res["yard_logits"] = _rel_max(ref32["logits"], ref["logits"])
            res["yard_loss"] = abs(ref32["loss"] - ref["loss"]) / abs(ref["loss"])
            res["yard_grads_global"] = yg
            res["yard_grads_own"] = yo
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
