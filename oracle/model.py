"""Functional CPU restatement of the reference's live training forward (sine2pi/ASR-model).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  PARITY UNPINNED (no reference fixtures exist;
executing the reference was denied).

Every function restates the cited reference lines with plain torch CPU ops.  Differences from the
reference, all deliberate and documented in DESIGN.md:
  * randomness is explicit: gumbel noise and dropout masks come from oracle/noise.py, addressed by
    (site key, logical index), so the HIP path can reproduce every draw;
  * the reference runs at batch 1 only (SURVEY.md §7 "Hard parts"); this oracle takes a batch and
    keeps batch-1 semantics per sample (BatchNorm statistics, MSheath's .item() control flow and
    rotary magnitudes are computed per sample; the loss is the mean over all non-pad tokens);
  * Dimensions.layer != 4 makes residual.router's Linear(3D, 3) fail in the reference
    (model.py:541, 563, 578); the oracle evaluates the router on 3 copies, which is what layer=4
    does (it is the identity up to rounding either way).

Parameters come as a name -> tensor dict using the reference's module-tree names
(e.g. "processor.block.0.attn.kv.1.weight").
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from . import keys as K
from . import noise as N

THETA = 30000.0


class Noise:
    """Keyed noise for one forward (seed, step); returns tensors in the oracle dtype."""

    def __init__(self, seed: int, step: int, dtype):
        self.seed, self.step, self.dtype = seed, step, dtype

    def key(self, site: str) -> int:
        return K.site_key(self.seed, self.step, site)

    def abby(self, site: str, sids, H: int, L: int) -> torch.Tensor:
        """(B, H, L, 3) gumbel noise for an AbbyNormal call on rows (sid, h, l)."""
        sid = np.asarray(sids, dtype=np.uint64)[:, None, None, None]
        h = np.arange(H, dtype=np.uint64)[None, :, None, None]
        l = np.arange(L, dtype=np.uint64)[None, None, :, None]
        k = np.arange(3, dtype=np.uint64)[None, None, None, :]
        idx = ((sid * np.uint64(H) + h) * np.uint64(K.LSTRIDE) + l) * np.uint64(3) + k
        return torch.from_numpy(N.gumbel(self.key(site), idx).astype(np.float64)).to(self.dtype)

    def policy(self, site: str, sids, layers: int) -> torch.Tensor:
        sid = np.asarray(sids, dtype=np.uint64)[:, None, None]
        i = np.arange(layers, dtype=np.uint64)[None, :, None]
        k = np.arange(3, dtype=np.uint64)[None, None, :]
        idx = (sid * np.uint64(64) + i) * np.uint64(3) + k
        return torch.from_numpy(N.gumbel(self.key(site), idx).astype(np.float64)).to(self.dtype)

    def keep(self, site: str, sids, C: int, T: int, p: float) -> torch.Tensor:
        """(B, C, T) dropout keep mask scaled by 1/(1-p) (nn.Dropout, train mode)."""
        sid = np.asarray(sids, dtype=np.uint64)[:, None, None]
        c = np.arange(C, dtype=np.uint64)[None, :, None]
        t = np.arange(T, dtype=np.uint64)[None, None, :]
        idx = (sid * np.uint64(C) + c) * np.uint64(K.LSTRIDE) + t
        u = N.uniform(self.key(site), idx)
        keep = (u >= np.float32(p)).astype(np.float64) / (1.0 - p)
        return torch.from_numpy(keep).to(self.dtype)


class Decisions:
    """Record / replay of the forward's hard decisions (keys as asrx/decisions.py):
      ("abby", key, sid) -> int64 (L, H) AbbyNormal mode index (gumbel argmax, essentials.py:170)
      ("ion", key, sid, layer) -> (L,) v_gate STthreshold output (model.py:330-334, 351)
      ("action", key, sid, layer) -> (action, forced) MSheath jump (model.py:476-482)
      ("cond", key, sid) -> bool (L, H, d) AbbyNormal mode 2's max > 2 avg per feature (rows in mode 2,
                            essentials.py:176-177)
    record: every decision taken is stored in `rec`.  replay: a decision found in `table` is used
    instead of the one this forward would take (the continuous values -- soft gumbel probabilities,
    STE paths -- are still this forward's own), so the oracle follows the HIP path's discrete
    trajectory and its gradients can be compared without decision flips."""

    def __init__(self, table=None):
        self.rec: dict = {}
        self.table = table
        self.replayed = 0
        self.overridden = 0
        self.cond_overridden = 0


_DEC: Decisions | None = None


def use_decisions(dec: Decisions | None):
    """Install (or remove, None) the decision recorder / replayer for the following forwards."""
    global _DEC
    _DEC = dec


def _decide_abby(index, dkey, heads: bool):
    """index: (B, L, 1) or (B, H, L, 1) argmax; dkey = (site key, sids)."""
    if _DEC is None or dkey is None:
        return index
    key, sids = dkey
    out = index.clone()
    for s, sid in enumerate(sids):
        got = index[s, ..., 0].t() if heads else index[s]  # (L, H)
        _DEC.rec[("abby", int(key), int(sid))] = got.clone()
        if _DEC.table is not None and ("abby", int(key), int(sid)) in _DEC.table:
            want = _DEC.table[("abby", int(key), int(sid))].to(index.dtype)
            _DEC.overridden += int((want != got).sum())
            _DEC.replayed += 1
            if heads:
                out[s, ..., 0] = want.t()
            else:
                out[s] = want
    return out


def _decide_cond(cond, index, dkey, heads: bool):
    """AbbyNormal mode 2's per-feature choice cond = max > 2 avg (essentials.py:176-177), (B, L, d) or
    (B, H, L, d) bool; index the (replayed) mode per row.  Recorded for the rows in mode 2 as (L, H, d);
    replayed from ("cond", key, sid) on the rows the replayed mode puts in mode 2."""
    if _DEC is None or dkey is None:
        return cond
    key, sids = dkey
    out = cond.clone()
    for s, sid in enumerate(sids):
        m1 = index[s, ..., 0] == 1  # (L,) or (H, L)
        own = cond[s] & m1.unsqueeze(-1)
        _DEC.rec[("cond", int(key), int(sid))] = (own.permute(1, 0, 2) if heads else own.unsqueeze(1)).clone()
        want = _DEC.table.get(("cond", int(key), int(sid))) if _DEC.table is not None else None
        if want is not None:
            want = (want.permute(1, 0, 2) if heads else want[:, 0, :]).to(cond.device)
            new = torch.where(m1.unsqueeze(-1), want, cond[s])
            _DEC.cond_overridden += int((new != cond[s]).sum())
            out[s] = new
    return out


# bf16 rounding emulation (conditioning measurements only, tools/bf16_sensitivity.py): the named points
# round their operands to bf16 in the forward (straight-through: the backward is the float64 one).
# Empty by default -- the oracle is the reference's arithmetic in the requested dtype.
EMU: set = set()


def _r(x, point):
    if point not in EMU:
        return x
    r = x.to(torch.bfloat16).to(x.dtype)
    if "x3" in EMU:
        # split-bf16 ("bf16x3") operands: hi = bf16(x), lo = bf16(x - hi); the 3-MFMA product
        # hi*hi + hi*lo + lo*hi sees x as hi + lo (the dropped lo*lo term is ~2^-16 of the product's ulp)
        r = r + (x - r).to(torch.bfloat16).to(x.dtype)
    return x + (r - x).detach()


class _RoundGrad(torch.autograd.Function):
    """Identity forward; the arriving gradient rounded to bf16 (the bf16 dY of a perf-mode backward GEMM)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _rg(x, point):
    """With "bwd" in EMU: the gradient arriving at x rounded to bf16 at an enabled point."""
    if point not in EMU or "bwd" not in EMU:
        return x
    return _RoundGrad.apply(x)


def _lin(P, name, x):
    b = P.get(name + ".bias")
    pt = "qkproj" if name.endswith((".q.1", ".kv.1")) else "lin"
    return _rg(F.linear(_r(x, pt), _r(P[name + ".weight"], pt), b), pt)


# ------------------------------------------------------------------------------- norms


def abby_normal(P, pre, x, g, dkey=None):
    """essentials.py:155-191 (AbbyNormal.forward, confidence=None).  g: gumbel noise, shape of
    the router logits.  dkey: (site key, sids) of the call for the decision recorder."""
    d = x.size(-1)
    size = max(3, int(d * 0.05))
    if size % 2 == 0:
        size += 1
    pad = size // 2
    div = x * x
    logits = _lin(P, pre + ".mode_router.2", F.silu(_lin(P, pre + ".mode_router.0", x)))
    mean_val = x.abs().mean(dim=-1, keepdim=True)
    std_val = x.std(dim=-1, keepdim=True)
    cv = std_val / (mean_val + 1e-6)
    # F.gumbel_softmax(logits + cv, tau=1, hard=True) with gumbels = g
    y_soft = torch.softmax(logits + cv + g, dim=-1)
    index = _decide_abby(y_soft.argmax(dim=-1, keepdim=True), dkey, x.dim() == 4)
    y_hard = torch.zeros_like(y_soft).scatter_(-1, index, 1.0)
    dec = y_hard - y_soft.detach() + y_soft
    rows = div.reshape(-1, 1, d)  # pooling runs along the feature axis (essentials.py:171-172)
    avg_d = F.avg_pool1d(rows, kernel_size=size, stride=1, padding=pad).reshape(div.shape)
    max_d = F.max_pool1d(rows, kernel_size=size, stride=1, padding=pad).reshape(div.shape)
    cond = _decide_cond(max_d > 2.0 * avg_d, index, dkey, x.dim() == 4).to(x.dtype)
    mode2 = cond * max_d + (1 - cond) * avg_d
    mode3 = avg_d
    div = dec[..., 0:1] * avg_d + dec[..., 1:2] * mode2 + dec[..., 2:3] * mode3
    denom = (div * 1e-4 + 1.0).pow(0.75)
    return x / denom


def abby_rows(P, pre, x, noise, site, sids):
    """AbbyNormal on (B, L, D) with noise rows (sid, l)."""
    g = noise.abby(site, sids, 1, x.shape[1])[:, 0]
    return abby_normal(P, pre, x, g, (noise.key(site), sids))


def channel_layer_norm(P, pre, x):
    """essentials.LayerNorm (essentials.py:110-113) on (B, C, T): normalise over channels."""
    y = F.layer_norm(x.transpose(1, -1), (x.shape[1],), P[pre + ".gamma"], P[pre + ".beta"], 1e-5)
    return y.transpose(1, -1)


def sinusoids(ctx, dims, dtype, theta=THETA):
    """essentials.py:354-358, evaluated in float32 like the reference."""
    tscales = torch.exp(-torch.log(torch.tensor(float(theta))) / (dims // 2 - 1)
                        * torch.arange(dims // 2, dtype=torch.float32))
    scaled = torch.arange(ctx, dtype=torch.float32).unsqueeze(1) * tscales.unsqueeze(0)
    return torch.cat([torch.sin(scaled), torch.cos(scaled)], dim=1).to(dtype)


# ------------------------------------------------------------------------------- encoder


def _weight_norm(g, v):
    return g * v / v.norm(dim=(1, 2), keepdim=True)


def _batch_norm_per_sample(y, P, pre, training, eps=1e-5):
    w, b = P[pre + ".weight"], P[pre + ".bias"]
    if not training:
        rm, rv = P[pre + ".running_mean"], P[pre + ".running_var"]
        return (y - rm[None, :, None]) / torch.sqrt(rv[None, :, None] + eps) * w[None, :, None] + b[None, :, None]
    out = []
    for s in range(y.shape[0]):  # batch-1 statistics (the reference trains at batch 1)
        ys = y[s:s + 1]
        mean = ys.mean(dim=(0, 2), keepdim=True)
        var = ys.var(dim=(0, 2), unbiased=False, keepdim=True)
        out.append((ys - mean) / torch.sqrt(var + eps) * w[None, :, None] + b[None, :, None])
    return torch.cat(out)


def encode_stream(P, x, layers, noise, sids, training, site="enc"):
    """AudioEncoder._process_feature (model.py:149-163) with ConvLite (model.py:109-118)."""
    if x.dim() == 2:
        x = x.unsqueeze(0)
    if x.shape[1] > 1:
        x = F.conv1d(x, P["enc.conv1.0.weight"], P["enc.conv1.0.bias"], padding=1)
    else:
        x = F.conv1d(x, P["enc.conv2.0.weight"], P["enc.conv2.0.bias"], padding=1)
    B, D, T = x.shape
    for l in range(layers):
        pre = f"enc.encoder.{l}"
        x = F.gelu(x)
        W = _weight_norm(P[pre + ".1.parametrizations.weight.original0"],
                         P[pre + ".1.parametrizations.weight.original1"])
        x = F.conv1d(x, W, P[pre + ".1.bias"], padding=1)
        x = channel_layer_norm(P, pre + ".2", x)
        res = x
        y = F.conv1d(x, P[pre + ".3.point1.weight"], P[pre + ".3.point1.bias"])
        y = F.glu(y, dim=1)
        y = F.conv1d(y, P[pre + ".3.depth.weight"], P[pre + ".3.depth.bias"], padding=7, groups=D)
        y = _batch_norm_per_sample(y, P, pre + ".3.bn", training)
        y = F.silu(y)
        y = F.conv1d(y, P[pre + ".3.point2.weight"], P[pre + ".3.point2.bias"])
        if training:
            y = y * noise.keep(f"{site}.L{l}.cl", sids, D, T, 0.1)
        x = res + y
        x = F.gelu(x)
        x = F.conv1d(x, P[pre + ".5.weight"], P[pre + ".5.bias"], padding=1, groups=D)
        x = F.gelu(x)
        if training:
            x = x * noise.keep(f"{site}.L{l}.dr", sids, D, T, 0.1)
    x = x.permute(0, 2, 1).contiguous()
    return x + sinusoids(T, D, x.dtype)


# ------------------------------------------------------------------------------- attention


def rotary_freqs(dims, head, masked: bool):
    """rotary.compute_f (model.py:191-196) with x=None, in float32 like the reference."""
    hd = dims // head
    if not masked:
        # essentials.gammatone (essentials.py:237-240): pow(40, linspace(0,1,hd/2)) * 200 / 1000
        scale = torch.pow(8000.0 / 200.0, torch.linspace(0, 1, hd // 2, dtype=torch.float32)) * 200.0
        scale = scale / 1000
        return 200 * scale / 1000
    return torch.arange(0, hd, 2, dtype=torch.float32) / hd * torch.log(torch.tensor(THETA))


def rotary(x, src, dims, head, masked):
    """rotary.forward (model.py:198-214), per sample: x (B, H, L, hd), src (B, L, D)."""
    L = x.shape[2]
    t = torch.arange(L, dtype=torch.float32)
    ang = torch.einsum("i,j->ij", t, rotary_freqs(dims, head, masked))  # float32 angles
    m = torch.norm(src, dim=-1, keepdim=True)  # (B, L, 1)
    ang = ang.to(x.dtype)
    fr, fi = m * torch.cos(ang)[None], m * torch.sin(ang)[None]  # (B, L, hd/2) = polar(m, ang)
    xr, xi = x[..., 0::2], x[..., 1::2]
    fr, fi = fr[:, None], fi[:, None]
    out = torch.empty_like(x)
    out[..., 0::2] = xr * fr - xi * fi
    out[..., 1::2] = xr * fi + xi * fr
    return out


def attention(P, pre, x, xa, masked, cfg, noise, site_q, sids_q, site_kv, sids_kv):
    """attention.forward (model.py:258-262, 302-307, 316-317), pt=None, pitch_bias=None."""
    D, H = cfg["dims"], cfg["head"]
    hd = D // H
    src = xa if xa is not None else x
    B, Lq, _ = x.shape
    Lk = src.shape[1]
    kvn = abby_rows(P, pre + ".kv.0", src, noise, site_kv + ".kv", sids_kv)
    kv = _lin(P, pre + ".kv.1", kvn)  # 'b c (kv h d) -> kv b h c d'
    k = kv[..., :D].reshape(B, Lk, H, hd).permute(0, 2, 1, 3)
    v = kv[..., D:].reshape(B, Lk, H, hd).permute(0, 2, 1, 3)
    qn = abby_rows(P, pre + ".q.0", x, noise, site_q + ".q", sids_q)
    q = _lin(P, pre + ".q.1", qn).reshape(B, Lq, H, hd).permute(0, 2, 1, 3)
    scale = hd ** -0.25
    q = q * scale
    k = k * scale
    q = rotary(q, x, D, H, masked)
    k = rotary(k, src, D, H, masked)
    gq = noise.abby(site_q + ".qh", sids_q, H, Lq)
    gk = noise.abby(site_kv + ".kh", sids_kv, H, Lk)
    q = abby_normal(P, pre + ".ln", q, gq, (noise.key(site_q + ".qh"), sids_q))
    k = abby_normal(P, pre + ".ln", k, gk, (noise.key(site_kv + ".kh"), sids_kv))
    s = _rg((_r(q, "qk") @ _r(k, "qk").transpose(-1, -2)) / math.sqrt(hd), "qk")  # bwd: dS rounded
    if masked:
        s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool).triu(1), float("-inf"))
    a = _rg(_r(torch.softmax(s, dim=-1), "pv") @ _r(v, "pv"), "pv")  # bwd: dO rounded
    a = a.permute(0, 2, 1, 3).reshape(B, Lq, D)
    return _lin(P, pre + ".out.1", a)


# ------------------------------------------------------------------------------- gates


def v_gate(P, pre, x, hard_override=None):
    """model.py:346-351 -> (ion, x_val).  hard_override: the thresholded value to use (replay)."""
    D = x.shape[-1]
    key = torch.softmax(F.normalize(x, p=2, dim=-1) @ F.normalize(P[pre + ".mkey"], p=2, dim=-1).t()
                        / math.sqrt(D), dim=-1)
    m = _lin(P, pre + ".mlp.2", F.silu(_lin(P, pre + ".mlp.0", x)))
    x_val = _lin(P, pre + ".concat", torch.cat((key @ P[pre + ".mval"], m), dim=-1))
    hard = (x_val > P[pre + ".tx"]).to(x.dtype)
    if hard_override is not None:
        hard = hard_override.to(x.dtype).reshape(hard.shape)
    ion = hard + (x_val - x_val.detach())  # STthreshold: binary forward, identity backward
    return ion, x_val


def _ln(P, pre, x):
    return F.layer_norm(x, (x.shape[-1],), P[pre + ".weight"], P[pre + ".bias"], 1e-5)


def msheath(P, pre, x, layer, g_pol, dkey=None):
    """MSheath.forward (model.py:429-507) at batch 1, run per sample.  g_pol: (B, layer, 3).
    dkey: (site key, sids) of the call for the decision recorder."""
    outs = []
    D = x.shape[-1]
    for s in range(x.shape[0]):
        xs = x[s:s + 1]
        ctx = xs.shape[1]
        orig_x = xs
        mem_w = P[pre + ".mem_w"].expand(1, -1, -1)
        pooled = xs.mean(dim=1)
        policy = torch.softmax(_lin(P, pre + ".pnet.net.2", F.silu(_lin(P, pre + ".pnet.net.0", pooled))), -1)
        i = 0
        while i < layer:
            lp = f"{pre}.layers.{i}"
            dk = None if (_DEC is None or dkey is None) else (int(dkey[0]), int(dkey[1][s]), i)
            rep = None
            if dk is not None and _DEC.table is not None and ("ion",) + dk in _DEC.table:
                rep = _DEC.table[("ion",) + dk]
            ion, x_val = v_gate(P, lp + ".v_gate", xs, rep)
            if dk is not None:
                own = (x_val > P[lp + ".v_gate.tx"]).to(x_val.dtype).reshape(-1)
                _DEC.rec[("ion",) + dk] = own.detach().clone()
                if rep is not None:
                    _DEC.replayed += 1
                    _DEC.overridden += int((rep.reshape(-1).to(own.dtype) != own).sum())
            mlayer = ion.expand(-1, ctx, D)
            px = _ln(P, lp + ".ln", xs)
            out = _lin(P, lp + ".adapter", px) if i % 2 == 0 else px
            g_val = torch.sigmoid(_lin(P, lp + ".gate.0", px))
            xs = xs + g_val * (out * mlayer)
            mem = xs.mean(dim=1, keepdim=True)
            mem_v = torch.sigmoid(_lin(P, pre + ".mem_gate.0", mem))
            mem_w = mem_v * mem_w + (1 - mem_v) * mem
            potential = ion.mean()
            jump_g = 1.0
            forced = bool(potential < 0.1 and i < layer - 1)
            want = None
            if dk is not None and _DEC.table is not None and ("action",) + dk in _DEC.table:
                want = _DEC.table[("action",) + dk]
            if want is not None:
                forced = want[1]
            if forced and i < layer - 1:
                action = 1
            elif i < layer - 1:
                ys = torch.softmax(policy + g_pol[s:s + 1, i], dim=-1)  # gumbel_softmax(policy, hard)
                idx = ys.argmax(dim=-1, keepdim=True)
                if want is not None:
                    idx = torch.full_like(idx, int(want[0]))
                jump = torch.zeros_like(ys).scatter_(-1, idx, 1.0) - ys.detach() + ys
                action = int(jump.argmax(dim=-1).item())
                jump_g = jump[0, action]
            else:
                action = 0
            if dk is not None:
                _DEC.rec[("action",) + dk] = (action, forced and i < layer - 1)
            if action > 0:
                i_next = min(i + action + 1, layer)
                jump_w = P[pre + ".jump_s"][min(action - 1, 2)]
                jump_i = jump_w * orig_x + (1 - jump_w) * mem_w.expand(-1, ctx, -1)
                xs = xs + jump_i * jump_g
                i = i_next
            else:
                xs = xs * jump_g
                i += 1
        gate = torch.sigmoid(_lin(P, pre + ".mlp_gate.0", xs))
        h = _lin(P, pre + ".mlp.2", F.silu(_lin(P, pre + ".mlp.0", _ln(P, pre + ".mlp_ln", xs))))
        outs.append(xs + gate * h)
    return torch.cat(outs)


def tgate(P, pre, x):
    """model.py:532-535 with num_types=3."""
    types = torch.softmax(_lin(P, pre + ".cs.0", x), dim=-1)
    ga = torch.stack([torch.sigmoid(_lin(P, f"{pre}.ga.{k}.0", x)) for k in range(3)], dim=-1)
    return torch.sum(ga * types.unsqueeze(2), dim=-1)


def router(P, pre, x, copies=3):
    """model.py:545-557 on `copies` stacked copies of x (identity up to rounding)."""
    stack = torch.stack([x] * copies, dim=-1)
    inp = stack.view(stack.shape[0], stack.shape[1], -1)
    top = _lin(P, pre + ".top", inp)
    types, indices = torch.topk(top, 2, dim=-1)
    typ = torch.zeros_like(top).scatter_(-1, indices, torch.softmax(types, dim=-1))
    soft = torch.softmax(_lin(P, pre + ".soft.0", inp), dim=-1)
    alpha = torch.sigmoid(P[pre + ".alpha"])
    w = alpha * typ + (1 - alpha) * soft
    return torch.sum(stack * w.unsqueeze(2), dim=-1)


def residual(P, i, x, cfg, noise, site, sids, xa=None, xa_site=None, xa_sids=None, masked=False):
    """residual.forward (model.py:576-583) for processor.block.{i}."""
    pre = f"processor.block.{i}"
    L = cfg["layer"]
    x = abby_rows(P, pre + ".ln", x, noise, site + ".ln0", sids)
    x = msheath(P, pre + ".jump", x, L, noise.policy(site + ".jump", sids, L), (noise.key(site + ".jump"), sids))
    h = abby_rows(P, pre + ".ln", x, noise, site + ".ln1", sids)
    x = router(P, pre + ".router", x) + attention(P, pre + ".attn", h, None, masked, cfg, noise,
                                                   site + ".sa", sids, site + ".sa", sids)
    if xa is not None:
        xa = xa + sinusoids(xa.shape[1], xa.shape[-1], xa.dtype)
        xa = abby_rows(P, pre + ".ln", xa, noise, xa_site + ".ln", xa_sids)
        xa = msheath(P, pre + ".jump", xa, L, noise.policy(xa_site + ".jump", xa_sids, L),
                     (noise.key(xa_site + ".jump"), xa_sids))
        h = abby_rows(P, pre + ".ln", x, noise, site + ".ln2", sids)
        x = x + attention(P, pre + ".attn", h, router(P, pre + ".router", xa), False, cfg, noise,
                          site + ".ca", sids, xa_site + ".ca", xa_sids)
    m = abby_rows(P, pre + ".ln", x, noise, site + ".mlp.ln0", sids)
    m = tgate(P, pre + ".mlp.1", m)
    m = F.gelu(_lin(P, pre + ".mlp.2", m))
    m = _lin(P, pre + ".mlp.4", m)
    m = abby_rows(P, pre + ".ln", m, noise, site + ".mlp.ln1", sids)
    return x + m


def forward(P, cfg, text_ids, labels=None, spectrogram=None, pitch=None, waveform=None,
            seed=0, step=0, training=True, dtype=torch.float64, live_only=False, seq=False):
    """Model.forward (model.py:654-672) + processor.forward (model.py:602-629).

    live_only: evaluate only the last block.  processor.forward restarts every block from the
    embedding `x` and only the last block's d / g reach the output (model.py:617-628), and the
    noise of a block is addressed by its own site keys, so skipping blocks 0..L-2 leaves logits,
    loss and every gradient unchanged (they only cost the reference compute and RNG draws).
    seq: processor(..., seq=True) (model.py:624-626, the generate path): out = g, no blend."""
    P = {k: v.to(dtype) if v.is_floating_point() else v for k, v in P.items()}
    noise = Noise(seed, step, dtype)
    L = cfg["layer"]
    streams = {"a": pitch, "b": spectrogram, "c": waveform}
    first = next(t for t in (pitch, spectrogram, waveform) if t is not None)
    B = first.shape[0]
    pick = {"a": ("a", "b", "c"), "b": ("b", "a", "c"), "c": ("c", "a", "b")}  # aborc (essentials.py:25)
    xa = {}
    for si, s in enumerate("abc"):
        src = next(streams[k] for k in pick[s] if streams[k] is not None)
        sids = [si * B + b for b in range(B)]
        xa[s] = encode_stream(P, src.to(dtype), L, noise, sids, training)
    sid_t = list(range(B))
    sids = {s: [si * B + b for b in range(B)] for si, s in enumerate("abc")}
    T = text_ids.shape[1]
    x = P["processor.token.weight"][text_ids] + P["processor.position"][:T]
    for i in (range(L - 1, L) if live_only else range(L)):
        a = residual(P, i, x, cfg, noise, f"b{i}.ta", sid_t, masked=True)
        A1 = residual(P, i, xa["a"], cfg, noise, f"b{i}.audio", sids["a"])
        b_ = residual(P, i, a, cfg, noise, f"b{i}.tb", sid_t, xa=A1, xa_site=f"b{i}.xa", xa_sids=sids["a"])
        A2 = residual(P, i, xa["b"], cfg, noise, f"b{i}.audio", sids["b"])
        c_ = residual(P, i, b_, cfg, noise, f"b{i}.tc", sid_t, xa=A2, xa_site=f"b{i}.xa", xa_sids=sids["b"])
        A3 = residual(P, i, xa["c"], cfg, noise, f"b{i}.audio", sids["c"])
        d = residual(P, i, c_, cfg, noise, f"b{i}.td", sid_t, xa=A3, xa_site=f"b{i}.xa", xa_sids=sids["c"])
        e = a + b_ + c_
        g = residual(P, i, d, cfg, noise, f"b{i}.tg", sid_t, xa=e, xa_site=f"b{i}.tg.xa", xa_sids=sid_t)
    if seq:
        x = g
    else:
        blend = torch.sigmoid(P["processor.blend"])
        x = blend * d + (1 - blend) * g
    x = abby_rows(P, "processor.ln", x, noise, "final.ln", sid_t)
    logits = _r(x, "logits") @ _r(P["processor.token.weight"], "logits").t()
    loss = None
    if labels is not None:
        loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index=0)
    return {"logits": logits, "loss": loss}


def generate(P, cfg, spectrogram=None, pitch=None, waveform=None, max_new_tokens=150, seed=0, step=0,
             dtype=torch.float64):
    """Model.generate (model.py:674-701): eval mode, the encoder on the audio streams, then per new
    token the processor with seq=True over the tokens so far (starting from BOS = 1), argmax of the
    last position, stop once every sequence emitted EOS = 2.  The whole forward is recomputed for every
    token exactly as the reference does (blocks 0..L-2 are skipped: they never reach the output, see
    forward(live_only)); the gumbel noise is the keyed noise of one (seed, step), the same for every
    decoding step."""
    first = next(t for t in (pitch, spectrogram, waveform) if t is not None)
    B = first.shape[0]
    y = torch.ones(B, 1, dtype=torch.long)
    with torch.no_grad():
        for _ in range(max_new_tokens):
            logits = forward(P, cfg, y, spectrogram=spectrogram, pitch=pitch, waveform=waveform, seed=seed,
                             step=step, training=False, dtype=dtype, live_only=True, seq=True)["logits"]
            nxt = logits[:, -1, :].argmax(dim=-1, keepdim=True)
            y = torch.cat((y, nxt), dim=1)
            if bool((nxt == 2).all()):
                break
    return y
