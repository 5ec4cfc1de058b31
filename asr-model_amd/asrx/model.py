"""MI355X-native Model with the reference's module tree, parameter names and forward signature
(model.py:631-672).  `Model(param).state_dict()` is key-compatible with the reference; the forward
runs the HIP kernels of csrc/ through asrx.ops.

Execution differs from the reference only where batch-1 semantics had to be generalised
(SURVEY.md §7 "Hard parts"): clips are batched with per-sample BatchNorm statistics, per-sample
MSheath control flow evaluated on device as masked compute (no .item() syncs), and keyed noise.
Activations are channels-last (B, T, D) throughout the encoder, so no permutes are needed.
Blocks 0..L-2 are computed faithfully (the reference recomputes them and discards the result,
model.py:617-628) under no_grad, since nothing downstream depends on them.
"""
from __future__ import annotations

import contextlib
import math

import torch
from torch import nn
from torch.nn.utils.parametrizations import weight_norm

from . import gemm as gemm_mod
from . import lib, ops, prec
from .config import Dimensions
from .noise import NoiseCtx

THETA = 30000.0

# ------------------------------------------------------------------------------- constant tables
_TABLES: dict = {}


def sinusoids(ctx: int, dims: int, device) -> torch.Tensor:
    """essentials.sinusoids (essentials.py:354-358), evaluated in float32 exactly like the reference
    and cached on the device."""
    key = ("pe", ctx, dims, str(device))
    if key not in _TABLES:
        tscales = torch.exp(-torch.log(torch.tensor(float(THETA))) / (dims // 2 - 1)
                            * torch.arange(dims // 2, dtype=torch.float32))
        scaled = torch.arange(ctx, dtype=torch.float32).unsqueeze(1) * tscales.unsqueeze(0)
        _TABLES[key] = _to_device(torch.cat([torch.sin(scaled), torch.cos(scaled)], dim=1).contiguous(), device)
    return _TABLES[key]


def _to_device(t, device):
    """A constant table, made once and then read from several streams: complete the copy before any
    stream can use it."""
    t = t.to(device)
    if t.is_cuda:
        torch.cuda.current_stream(t.device).synchronize()
    return t


def rotary_freqs(dims: int, head: int, masked: bool, device) -> torch.Tensor:
    """rotary.compute_f (model.py:191-196) with x=None, float32 like the reference."""
    key = ("rot", dims, head, masked, str(device))
    if key not in _TABLES:
        hd = dims // head
        if not masked:
            scale = torch.pow(8000.0 / 200.0, torch.linspace(0, 1, hd // 2, dtype=torch.float32)) * 200.0
            scale = scale / 1000  # essentials.gammatone
            f = 200 * scale / 1000
        else:
            f = torch.arange(0, hd, 2, dtype=torch.float32) / hd * torch.log(torch.tensor(THETA))
        _TABLES[key] = _to_device(f.contiguous(), device)
    return _TABLES[key]


# ------------------------------------------------------------------------------- norms


class AbbyNormal(nn.Module):
    """essentials.AbbyNormal (essentials.py:140-191)."""

    def __init__(self, dims, size: int = 5, alpha: float = 1e-4, beta: float = 0.75, k: float = 1.0,
                 threshold: float = 0.8):
        super().__init__()
        self.size, self.alpha, self.beta, self.k, self.tx = size, alpha, beta, k, threshold
        self.mode_router = nn.Sequential(nn.Linear(dims, dims), nn.SiLU(), nn.Linear(dims, 3))

    def run(self, x, noise: NoiseCtx, site: str, sid_base: int, L: int, H: int = 1, out_bf16: bool = False,
            tgate=None, residual=None):
        """out_bf16: the output only feeds GEMM / attention operands (stored bf16 in perf mode); tgate: the
        consuming tgate (its cs Linear(d, 3) is evaluated inside the norm's kernel); residual: returns
        residual + AbbyNormal(x) (the add fused into the norm's kernel in perf mode)."""
        return ops.abby_normal(self, x, L, H, sid_base, noise.key(site), True, out_bf16, tgate, residual)


class LayerNorm(nn.Module):
    """essentials.LayerNorm (essentials.py:102-113): layer_norm over channels."""

    def __init__(self, dims, eps=1e-5):
        super().__init__()
        self.dims, self.eps = dims, eps
        self.gamma = nn.Parameter(torch.ones(dims))
        self.beta = nn.Parameter(torch.zeros(dims))


def get_norm(n_type: str, dims: int):
    if n_type != "AbbyNormal":
        raise NotImplementedError(f"n_type {n_type!r}: only the reachable 'AbbyNormal' path is built "
                                  "(SURVEY.md §2 #10)")
    return AbbyNormal(dims, size=5, alpha=1e-4, beta=0.75, k=1.0, threshold=0.8)


def get_activation(act: str) -> nn.Module:
    if act != "gelu":
        raise NotImplementedError(f"act {act!r}: only 'gelu' (the configured activation) is built")
    return nn.GELU()


# ------------------------------------------------------------------------------- encoder


class ConvLite(nn.Module):
    def __init__(self, dims, kernel_size=15):
        super().__init__()
        self.point1 = nn.Conv1d(dims, dims * 2, kernel_size=1)
        self.glu = nn.GLU(dim=1)
        self.depth = nn.Conv1d(dims, dims, kernel_size=kernel_size, padding=(kernel_size - 1) // 2, groups=dims)
        self.bn = nn.BatchNorm1d(dims)
        self.swish = nn.SiLU()
        self.point2 = nn.Conv1d(dims, dims, kernel_size=1)
        self.dropout = nn.Dropout(0.1)

    def run(self, x, noise: NoiseCtx, site: str, sid_base: int):
        """model.py:109-118 on channels-last (B, T, D)."""
        D = x.shape[-1]
        x = ops.fork(x)  # read by point1 and the residual add
        res = x
        y = ops.linear(x, self.point1.weight, self.point1.bias)  # (2D, D, 1) leaf: gradient straight into it
        y = ops.glu(y)
        y = ops.DWConv.apply(y, self.depth.weight, self.depth.bias)
        if self.training:
            stats = []
            y = ops.BatchNormPS.apply(y, self.bn.weight, self.bn.bias, self.bn.eps, stats)
            self._update_running(stats[0], y.shape[1])
        else:
            y = ops.batch_norm_eval(y, self.bn.weight, self.bn.bias, self.bn.running_mean, self.bn.running_var,
                                    self.bn.eps)
        y = ops.act(y, "silu")
        y = ops.linear(y, self.point2.weight, self.point2.bias)
        if self.training:  # res + dropout(y) in one pass
            return ops.dropout_add(res, y, sid_base, noise.key(site + ".cl"), 0.1)
        return ops.add(res, y)

    @torch.no_grad()
    def _update_running(self, stats, T):
        # batch-1 semantics: one update per clip would be applied by the reference; here the mean of
        # the per-clip statistics is applied once per stream group (running stats do not affect the
        # train-mode output).  One kernel (asrx_bn_running) instead of the ATen update chain.
        mean, rstd = stats
        B, C = mean.shape
        bn = self.bn
        lib.call("asrx_bn_running", lib.ptr(mean), lib.ptr(rstd), lib.ptr(bn.running_mean), lib.ptr(bn.running_var),
                 lib.ptr(bn.num_batches_tracked), B, C, T, float(bn.eps), float(bn.momentum), lib.stream())


class AudioEncoder(nn.Module):
    """model.py:120-169 (norm=False, enc=False)."""

    def __init__(self, mels, dims, head, layer, act, n_type, norm=False, enc=False):
        super().__init__()
        if norm or enc:
            raise NotImplementedError("AudioEncoder(norm/enc=True) is not reachable from Model")
        self.norm = nn.Identity()
        self.local_norm = nn.Identity()
        act_fn = get_activation(act)
        self.conv1 = nn.Sequential(nn.Conv1d(mels, dims, kernel_size=3, stride=1, padding=1), self.norm)
        self.conv2 = nn.Sequential(nn.Conv1d(1, dims, kernel_size=3, stride=1, padding=1), self.local_norm)
        self.EncoderLayer = nn.Identity()
        self.encoder = nn.ModuleList()
        for _ in range(layer):
            self.encoder.append(nn.Sequential(
                act_fn, weight_norm(nn.Conv1d(dims, dims, kernel_size=3, padding=1)),
                LayerNorm(dims),
                ConvLite(dims, kernel_size=15),
                act_fn,
                nn.Conv1d(dims, dims, kernel_size=3, stride=1, padding=1, groups=dims), act_fn, nn.Dropout(0.1)))

    def stem(self, x, out=None):
        """(B, C, T) -> (B, T, D): Conv1d(mels, D, 3) for C > 1, Conv1d(1, D, 3) otherwise (model.py:150-155)."""
        if x.dim() == 2:
            x = x.unsqueeze(0)
        B, C, T = x.shape
        if C > 1:
            xt = x.transpose(1, 2).contiguous()
            return ops.conv3(xt, self.conv1[0], out=out)
        return ops.Stem1.apply(x.reshape(B, T), self.conv2[0].weight, self.conv2[0].bias, out)

    def layers(self, x, noise: NoiseCtx, sid_base: int):
        n = len(self.encoder)
        fused_lead = False  # the previous layer's fused tail already applied this layer's leading GELU
        for l, layer in enumerate(self.encoder):
            if not fused_lead:
                x = ops.act(x, "gelu")
            fused_lead = False
            x = ops.conv3(x, layer[1])
            x = ops.layer_norm(x, layer[2].gamma, layer[2].beta, layer[2].eps)
            x = layer[3].run(x, noise, f"enc.L{l}", sid_base)
            x = ops.act(x, "gelu")
            x = ops.DWConv.apply(x, layer[5].weight, layer[5].bias)
            if self.training:  # GELU -> Dropout(0.1) [-> next layer's GELU] in one kernel each way
                fused_lead = l + 1 < n
                x = ops.act_dropout(x, "gelu", sid_base, noise.key(f"enc.L{l}.dr"), 0.1,
                                         "gelu" if fused_lead else "none")
            else:
                x = ops.act(x, "gelu")
        return ops.add_rows(x, sinusoids(x.shape[1], x.shape[2], x.device))

    def encode(self, streams, noise: NoiseCtx, B: int):
        """streams: list of 3 (B, C, T) tensors (a, b, c).  Returns 3 (B, T, D) encodings; streams
        of equal length share one batched pass (sample ids stay s*B + b)."""
        # runs of consecutive equal-length streams share one pass: their stems write straight into the
        # row blocks of one group buffer (no concatenation copy)
        lens = [s.shape[-1] for s in streams]
        out = [None] * len(streams)
        i = 0
        while i < len(streams):
            j = i + 1
            while j < len(streams) and lens[j] == lens[i]:
                j += 1
            if j == i + 1:
                x = self.stem(streams[i])
            else:
                Bs = [s.shape[0] if s.dim() == 3 else 1 for s in streams[i:j]]
                buf = torch.empty(sum(Bs), lens[i], self.conv1[0].weight.shape[0], device=streams[i].device)
                parts, r0 = [], 0
                for s, b in zip(streams[i:j], Bs):
                    parts.append(self.stem(s, out=buf[r0:r0 + b]))
                    r0 += b
                x = ops.join_group(buf, parts)
            y = self.layers(x, noise, i * B)
            out[i:j] = ops.split_rows(y, j - i)
            i = j
        return out


# ------------------------------------------------------------------------------- attention


class rotary(nn.Module):  # noqa: N801  (reference class name, model.py:171)
    def __init__(self, dims, head):
        super().__init__()
        self.head_dim = dims // head
        self.head = head
        self.dims = dims
        self.lin = nn.Linear(dims, self.head_dim // 2, bias=True)  # constructed, unused (model.py:178)


class attention(nn.Module):  # noqa: N801
    """model.py:234-317 (live path: pt=None, pitch_bias=None, modal=False)."""

    def __init__(self, dims, head, layer, n_type=None, modal=False):
        super().__init__()
        self.layer = layer
        self.head = head
        self.scale = (dims // head) ** -0.25
        self.modal = modal
        self.q = nn.Sequential(get_norm(n_type, dims), nn.Linear(dims, dims), nn.Identity())
        self.kv = nn.Sequential(get_norm(n_type, dims), nn.Linear(dims, dims * 2), nn.Identity())
        self.c = nn.Sequential(get_norm(n_type, dims), nn.Linear(dims, dims), nn.Identity())
        self.out = nn.Sequential(nn.Identity(), nn.Linear(dims, dims))
        self.conv = nn.Identity()
        self.ln = get_norm(n_type, dims // head)
        self.rot = rotary(dims, head)

    def project_kv(self, src, noise, site, sid_base, masked):
        """k, v of `src` (model.py:261, 304, 306-307 k-side): AbbyNormal -> Linear(D, 2D) split
        '(kv h d)' -> k: scale + rotary(|src|) + per-head AbbyNormal."""
        B, L, D = src.shape
        H, hd = self.head, D // self.head
        src = ops.want_rownorm(ops.fork(src))  # read by the kv AbbyNormal and rotary's |src|
        kvn = self.kv[0].run(src, noise, site + ".kv", sid_base, L, out_bf16=True)
        k, v = ops.kv_proj_rotary(kvn, self.kv[1].weight, self.kv[1].bias, src,
                                  rotary_freqs(D, H, masked, src.device), hd, self.scale)
        k = self.ln.run(k.view(B, L, H, hd), noise, site + ".kh", sid_base, L, H, out_bf16=prec.attn_bf16_io())
        vh = v.view(B, L, H, hd)
        if ops.sink_of(v) is not None:  # v is bf16-stored: attention adds its gradient into v's sink
            vh._asrx_sink = ops.sink_of(v)
        return k, vh

    def project_q(self, x, noise, site, sid_base, masked):
        B, L, D = x.shape
        H, hd = self.head, D // self.head
        qn = self.q[0].run(ops.want_rownorm(x), noise, site + ".q", sid_base, L, out_bf16=True)
        q = ops.linear_rotary(qn, self.q[1].weight, self.q[1].bias, x, rotary_freqs(D, H, masked, x.device), hd,
                              self.scale)
        return self.ln.run(q.view(B, L, H, hd), noise, site + ".qh", sid_base, L, H, out_bf16=prec.attn_bf16_io())

    def run(self, x, kv, noise, site, sid_base, masked, residual=None):
        """x: attention input (B, Lq, D); kv: None (self attention on x) or (k, v) of the cross
        source.  Returns the out-projected (B, Lq, D), plus `residual` when given (the residual add
        of model.py:578-580 fused into the out projection's epilogue)."""
        B, L, D = x.shape
        x = ops.fork(x)  # read by the q (and, self-attention, kv) AbbyNormal and rotary's |x|
        if kv is None:
            kv = self.project_kv(x, noise, site, sid_base, masked)
        q = self.project_q(x, noise, site, sid_base, masked)
        # o feeds only the out projection, which rounds it to bf16 anyway -- but when a backward runs,
        # the attention backward's Delta = rowsum(dO * o) needs o at fp32: dS = P (dP - Delta) subtracts
        # two nearly equal terms when the values barely vary over the keys, and a bf16 o turned that
        # cancellation into errors of several times the largest parameter gradient (tools/
        # debug_storage_grad.py).  So o is stored bf16 only without a backward (dead blocks, eval).
        o = ops.attention(q, kv[0], kv[1], masked, out_bf16=not ops._grad_needed(q, kv[0], kv[1]),
                          merge_heads=True)
        if residual is not None:
            return ops.linear_residual(residual, o, self.out[1].weight, self.out[1].bias)
        return ops.linear(o, self.out[1].weight, self.out[1].bias)  # o: (B, L, D), heads merged


# ------------------------------------------------------------------------------- MSheath


class AdaptiveSpan(nn.Module):
    """essentials.AdaptiveSpan (essentials.py:1219-1280): constructed by MSheath but never called;
    kept for parameter-name compatibility (span_scale)."""

    def __init__(self, dims, head, max_dist, sharpen=True, temp_scale=0.01):
        super().__init__()
        self.dims, self.head, self.max_dist = dims, head, max_dist
        self.sharpen, self.temp_scale = sharpen, temp_scale
        self.span_scale = nn.Parameter(torch.tensor(1.0))


class v_gate(nn.Module):  # noqa: N801  (model.py:336-358)
    def __init__(self, dims, mem=64, thresh=0.5):
        super().__init__()
        self.mkey = nn.Parameter(torch.randn(mem, dims))
        self.mval = nn.Parameter(torch.randn(mem, 1))
        self.mlp = nn.Sequential(nn.Linear(dims, dims // 2), nn.SiLU(), nn.Linear(dims // 2, 1))
        self.tx = nn.Parameter(torch.tensor(thresh, dtype=torch.float32), requires_grad=False)
        self.concat = nn.Linear(2, 1)


class MPNet(nn.Module):
    def __init__(self, dims, jump=2):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dims, 128), nn.SiLU(), nn.Linear(128, jump + 1))


class MSheath(nn.Module):
    """model.py:387-507."""

    def __init__(self, dims, head, layer, mini_hc=False, rate=2):
        super().__init__()
        if mini_hc:
            raise NotImplementedError("MSheath(mini_hc=True) is not reachable from residual")
        self.layer = layer
        self.dims = dims
        self.l_jump = True
        self.jstat = {0: 0, 1: 0, 2: 0}
        self.shared_head = AdaptiveSpan(dims, head, max_dist=1)
        self.mem_w = nn.Parameter(torch.zeros(1, 1, dims), requires_grad=True)
        self.mem_gate = nn.Sequential(nn.Linear(dims, 1), nn.Sigmoid())
        self.jump_s = nn.Parameter(torch.tensor([0.1, 0.05, 0.01]), requires_grad=True)
        self.layers = nn.ModuleList()
        for i in range(layer):
            self.layers.append(nn.ModuleDict({
                "ln": nn.LayerNorm(dims),
                "gate": nn.Sequential(nn.Linear(dims, 1), nn.Sigmoid()),
                "v_gate": v_gate(dims, mem=64, thresh=0.3),
                "adapter": nn.Linear(dims, dims) if i % 2 == 0 else None,
                "ranvier": None,
            }))
        self.pnet = MPNet(dims, jump=2)
        self.mlp_gate = nn.Sequential(nn.Linear(dims, 1), nn.Sigmoid())
        self.mlp = nn.Sequential(nn.Linear(dims, dims * 4), nn.SiLU(), nn.Linear(dims * 4, dims))
        self.mlp_ln = nn.LayerNorm(dims)

    # fused: one autograd node per call with a hand-written backward (asrx/msheath.py); False runs the
    # per-op composition below (same kernels and results; kept as the reference implementation of it)
    fused = True

    def run(self, x, noise: NoiseCtx, site: str, sid_base: int):
        """Batched MSheath.forward with batch-1 semantics per sample: every sample follows its own
        layer/jump trajectory, evaluated as masked compute on device (no host syncs)."""
        from . import msheath as _ms

        if self.fused and ops.DIRECT and _ms.supported(self, x.shape[-1]):
            gpol = ops.policy_noise(x.shape[0], self.layer, sid_base, noise.key(site), x.device)
            return _ms.msheath(self, x, gpol, tag=(noise.key(site), sid_base))
        return self.run_composed(x, noise, site, sid_base)

    def run_composed(self, x, noise: NoiseCtx, site: str, sid_base: int):
        B, L, D = x.shape
        dev = x.device
        orig = x
        mem_w = self.mem_w.reshape(1, D).expand(B, D).contiguous()
        pooled = ops.seg_mean(x)
        h = ops.linear(pooled, self.pnet.net[0].weight, self.pnet.net[0].bias, act="silu")
        policy = torch.softmax(ops.small_linear(h, self.pnet.net[2].weight, self.pnet.net[2].bias), dim=-1)
        gpol = ops.policy_noise(B, self.layer, sid_base, noise.key(site), dev)
        next_i = torch.zeros(B, device=dev)
        for i in range(self.layer):
            lay = self.layers[i]
            ion = ops.v_gate(lay["v_gate"], x)  # (B, L)
            px = ops.layer_norm(x, lay["ln"].weight, lay["ln"].bias, lay["ln"].eps)
            out = ops.linear(px, lay["adapter"].weight, lay["adapter"].bias) if lay["adapter"] is not None else px
            g_val = ops.small_linear(px, lay["gate"][0].weight, lay["gate"][0].bias, act="sigmoid")  # (B, L, 1)
            x_new = ops.AxpyRow2.apply(x, g_val.reshape(B, L), ion, out)
            mem = ops.seg_mean(x_new)
            mem_v = ops.small_linear(mem, self.mem_gate[0].weight, self.mem_gate[0].bias, act="sigmoid")  # (B, 1)
            alpha, beta, gam, mem_w, active, next_i = ops.MSheathCtrl.apply(
                policy, gpol[:, i], ion, mem_v.reshape(B), mem_w, mem, self.jump_s, next_i, i, self.layer)
            x = ops.JumpSelect.apply(x_new, orig, x, active, alpha, beta, gam)
        gate = ops.small_linear(x, self.mlp_gate[0].weight, self.mlp_gate[0].bias, act="sigmoid")
        hh = ops.layer_norm(x, self.mlp_ln.weight, self.mlp_ln.bias, self.mlp_ln.eps)
        hh = ops.linear(hh, self.mlp[0].weight, self.mlp[0].bias, act="silu")
        hh = ops.linear(hh, self.mlp[2].weight, self.mlp[2].bias)
        return ops.axpy_row(x, gate.reshape(B, L).contiguous(), hh)


# ------------------------------------------------------------------------------- blocks


class tgate(nn.Module):  # noqa: N801  (model.py:525-535)
    def __init__(self, dims, num_types=2):
        super().__init__()
        self.ga = nn.ModuleList([nn.Sequential(nn.Linear(dims, dims), nn.Sigmoid()) for _ in range(num_types)])
        self.cs = nn.Sequential(nn.Linear(dims, num_types), nn.Softmax(dim=-1))


class router(nn.Module):  # noqa: N801  (model.py:537-557)
    """Parameters kept for state_dict compatibility.  router(x, x, x) = sum_k w_k x with
    sum_k w_k = 1, i.e. the identity (up to one rounding), so the HIP path applies it as identity
    (tests/test_gpu_model.py checks it against the oracle's full evaluation)."""

    def __init__(self, dims, num_types):
        super().__init__()
        self.num_types = num_types
        self.top = nn.Linear(dims * num_types, num_types)
        self.soft = nn.Sequential(nn.Linear(dims * num_types, num_types), nn.Softmax(dim=-1))
        self.alpha = nn.Parameter(torch.ones(1), requires_grad=True)


class residual(nn.Module):  # noqa: N801  (model.py:559-583)
    def __init__(self, dims, head, layer, act, n_type, num_types=3):
        super().__init__()
        self.layer = layer - 1
        self.ln = get_norm(n_type=n_type, dims=dims)
        self.act_fn = get_activation(act)
        self.attn = attention(dims, head, layer, n_type=n_type)
        self.router = router(dims, num_types=num_types)
        self.jump = MSheath(dims, head, layer)
        self.mlp = nn.Sequential(self.ln, tgate(dims, num_types=num_types),
                                 nn.Linear(dims, dims * num_types), get_activation(act),
                                 nn.Linear(dims * num_types, dims), self.ln)

    def call(self, x, noise: NoiseCtx, site: str, sid_base: int, kv=None, masked=False):
        """residual.forward with the cross source given as precomputed (k, v) (see xa_side)."""
        L = x.shape[1]
        h = self.ln.run(x, noise, site + ".ln0", sid_base, L)
        x = ops.fork(self.jump.run(h, noise, site + ".jump", sid_base))  # each x: an AbbyNormal + an add
        h = self.ln.run(x, noise, site + ".ln1", sid_base, L)
        x = ops.fork(self.attn.run(h, None, noise, site + ".sa", sid_base, masked, residual=x))
        if kv is not None:
            h = self.ln.run(x, noise, site + ".ln2", sid_base, L)
            x = ops.fork(self.attn.run(h, kv, noise, site + ".ca", sid_base, False, residual=x))
        m = self.ln.run(x, noise, site + ".mlp.ln0", sid_base, L, out_bf16=True, tgate=self.mlp[1])
        m = ops.tgate(self.mlp[1], m, out_bf16=True)
        m = ops.linear(m, self.mlp[2].weight, self.mlp[2].bias, act="gelu", out_bf16=True)
        m = ops.linear(m, self.mlp[4].weight, self.mlp[4].bias)
        return self.ln.run(m, noise, site + ".mlp.ln1", sid_base, L, residual=x)  # x + mlp(x), model.py:583

    def xa_side(self, xa, noise: NoiseCtx, site: str, sid_base: int):
        """The cross source of residual.forward (model.py:579-582): xa + PE -> AbbyNormal -> MSheath
        -> attention k/v projection."""
        S, D = xa.shape[1], xa.shape[2]
        xa = ops.add_rows(xa, sinusoids(S, D, xa.device))
        xa = self.ln.run(xa, noise, site + ".ln", sid_base, S)
        xa = self.jump.run(xa, noise, site + ".jump", sid_base)
        return self.attn.project_kv(xa, noise, site + ".ca", sid_base, False)


class processor(nn.Module):  # noqa: N801  (model.py:585-629)
    def __init__(self, tokens, mels, dims, head, layer, act, n_type, ctx=2048):
        super().__init__()
        self.dims = dims
        self.ln = get_norm(n_type, dims)
        self.token = nn.Embedding(tokens, dims)
        self.pitch_tokens = nn.Embedding(1024, dims)
        self.position = nn.Parameter(torch.ones(ctx, dims), requires_grad=True)
        self.blend = nn.Parameter(torch.tensor(0.5), requires_grad=True)
        self.block = nn.ModuleList([residual(dims, head, layer, act, n_type) for _ in range(layer)])
        # Blocks 0..L-2 restart from the embeddings and never reach the output (model.py:617-628).
        # False (default): computed anyway, like the reference (faithful work).  True: skipped --
        # output-identical (keyed noise: no RNG stream to keep in step), reported separately.
        self.skip_dead_blocks = False
        # Dead blocks carry no autograd state, so their text side (8192-row calls at the tiny config:
        # launch-latency-bound kernels) runs on a second HIP stream under the next blocks' audio side
        # (bandwidth-bound, 192k-row calls).  Scheduling only: same kernels, same results.
        self.concurrent_dead_text = True
        # All of blocks 0..L-2 on two side streams (their audio and text sides), concurrently with the live
        # block's forward AND backward, joined at the end of the backward (round 4); False: the round-3
        # schedule above (dead audio on the current stream, dead text beside it, joined per forward)
        self.concurrent_dead_blocks = True
        # where the concurrent dead blocks are enqueued: "start" (before the live block: they share the GPU with
        # the live forward), "mid" (after the live audio side: beside the live text side, the cross entropy and
        # the backward) or "end" (after the live forward: beside the cross entropy and the backward)
        self.dead_blocks_at = "end"  # measured: end 5108-5111, mid 5097-5114, start 5061-5072 audio-s/s (profiles/r05_dead_at_ab.txt)
        # Opt-in: the concurrent dead blocks replayed from HIP graphs, one set per step signature (shapes,
        # grouping, precision switches, the bulk bf16 arena), so their launches cost one graph launch of host time
        # instead of ~30-45 us of Python each.  Same kernels, same shapes, same work; the replays reuse the capture
        # step's noise keys -- the dead blocks' outputs never reach the loss (model.py:617-628).  Off by default:
        # the steps it was built for turned out GPU-bound, not host-bound, and the replays run the side streams'
        # kernels with less overlap than eager launches (profiles/r06_host_vs_gpu.txt: small B = 8 452 vs 418 ms
        # per step, tiny B = 32 180 vs 180 ms, with the forward's host time 30 vs 260 ms and 18 vs 47 ms).
        self.graph_dead_blocks = False
        self.graph_dead_max = 4  # graphs kept per processor (each holds its own memory pool)
        self._dgraphs = {}
        self._dseen = set()
        self.keep_dead_out = False  # tests: dead_out = the last dead block's output (graph vs eager)
        self.dead_out = None
        self._side = None
        self._pending = None
        self._hold = []

    def forward(self, x, xa, noise: NoiseCtx, seq=False, features=False):
        """features: return the final norm's output instead of the tied logits (Model.forward then runs
        the logits fused with the cross entropy, ops.logits_ce)."""
        B, T = x.shape
        self.join_dead_blocks()  # a previous forward's side work (no backward ran since)
        xe = ops.Embedding.apply(x, self.token.weight)
        x = ops.add_rows(xe, self.position)
        A_in = [xa["a"], xa["b"], xa["c"]]
        nblk = len(self.block)
        live = nblk - 1
        cuda = x.is_cuda
        conc_dead = not self.skip_dead_blocks and live > 0 and cuda and self.concurrent_dead_blocks
        if conc_dead and self.dead_blocks_at == "start":
            self._enqueue_dead(live, x, xe, A_in, noise, B)
        elif not conc_dead:
            side = None
            keep = []  # cross-stream inputs stay referenced until the side stream is joined
            for i in range(live):
                if self.skip_dead_blocks:
                    break
                conc = self.concurrent_dead_text and cuda
                if conc and side is None:
                    side = self._side_streams(x.device)[1]
                    side.wait_stream(torch.cuda.current_stream())
                with torch.no_grad() if torch.is_grad_enabled() else contextlib.nullcontext():
                    self._dead_block(i, x, A_in, noise, B, None, side, keep)
            if side is not None:
                torch.cuda.current_stream().wait_stream(side)
            keep.clear()
        blk = self.block[live]
        a = ops.fork(blk.call(x, noise, f"b{live}.ta", 0, masked=True))
        A = self._audio(blk, A_in, noise, f"b{live}.audio", B, "call")
        KV = self._audio(blk, A, noise, f"b{live}.xa", B, "xa")
        if conc_dead and self.dead_blocks_at == "mid":  # after the live audio side, beside its text side
            self._enqueue_dead(live, x, xe, A_in, noise, B)
        b_ = ops.fork(blk.call(a, noise, f"b{live}.tb", 0, kv=KV[0]))
        c_ = ops.fork(blk.call(b_, noise, f"b{live}.tc", 0, kv=KV[1]))
        d = ops.fork(blk.call(c_, noise, f"b{live}.td", 0, kv=KV[2]))
        e = ops.add(a, b_, c_)
        kve = blk.xa_side(e, noise, f"b{live}.tg.xa", 0)
        g = blk.call(d, noise, f"b{live}.tg", 0, kv=kve)
        if conc_dead and self.dead_blocks_at == "end":
            self._enqueue_dead(live, x, xe, A_in, noise, B)
        if seq:
            out = g
        else:
            out = ops.blend(d, g, self.blend)  # sigmoid(blend) d + (1 - sigmoid(blend)) g
        out = self.ln.run(out, noise, "final.ln", 0, T, out_bf16=True)
        if features:
            return out
        return ops.linear(out, self.token.weight)

    def _enqueue_dead(self, live, x, xe, A_in, noise, B):
        """Blocks 0..L-2 depend on nothing but the embeddings and the encoder outputs (every block restarts
        from them) and nothing depends on them: they run on side streams, concurrently with the rest of the
        step, and are joined at the end of the backward (Model.forward's hook) -- or right away without one.
        Scheduling only: keyed noise, same kernels, same results."""
        main = torch.cuda.current_stream()
        s_audio, s_text = self._side_streams(x.device)
        if self._replay_dead(live, x, A_in, noise, B, main, s_audio, s_text):
            self._pending = (s_audio, s_text, [x, xe] + A_in, main)
            return
        s_audio.wait_stream(main)
        s_text.wait_stream(main)
        with torch.no_grad():
            for i in range(live):
                g = self._dead_block(i, x, A_in, noise, B, s_audio, s_text)
        if self.keep_dead_out:
            self.dead_out = g
        self._pending = (s_audio, s_text, [x, xe] + A_in, main)

    def _dead_signature(self, live, x, A_in, groups, B):
        from . import msheath
        return (live, tuple(x.shape), x.dtype, tuple((tuple(a.shape), a.dtype) for a in A_in), tuple(groups), B,
                str(x.device), prec.state(), self.training, ops.ROT_FUSED, ops.DIRECT, MSheath.fused,
                msheath.DETERMINISTIC, gemm_mod._nj_override, gemm_mod.plan_token())

    def _replay_dead(self, live, x, A_in, noise, B, main, s_audio, s_text):
        """Blocks 0..L-2 from the signature's HIP graphs (see graph_dead_blocks).  False: run them eagerly
        (graphs off, a first sighting, decisions recorded or kernels probed -- both need eager launches --, or
        the graph budget spent).

        Three graphs keep the eager schedule's two side streams: the text self calls of every dead block on
        s_text, the audio sides (self calls and cross k / v) on s_audio, then -- after an event on the audio
        graph -- the text cross calls on s_text.  One graph per stream, so no captured fork / join (whose
        branches the replay maps onto one hardware queue, profiles/r05_eager_vs_graph.txt): the 2048-8192-row
        text-side kernels keep running beside the audio side's 48k-192k-row ones."""
        from . import decisions, probe
        if (not self.graph_dead_blocks or self.graph_dead_max <= 0 or decisions.active() or probe.active()
                or torch.cuda.is_current_stream_capturing()):
            return False
        groups, i = [], 0  # runs of equal-length streams, batched as processor._audio batches them
        while i < len(A_in):
            j = i + 1
            while j < len(A_in) and A_in[j].shape[1] == A_in[i].shape[1]:
                j += 1
            groups.append((i, j))
            i = j
        sig = self._dead_signature(live, x, A_in, groups, B)
        ent = self._dgraphs.get(sig)
        if ent is None:
            # capture on a signature's second sighting -- or on its first once the bulk bf16 arena exists, when the
            # live forward ran first (its tables and lazy buffers then exist; bench.py's warm-up steps capture)
            ready = sig in self._dseen or (sig[-1] is not None and self.dead_blocks_at == "end")
            self._dseen.add(sig)
            if not ready or len(self._dgraphs) >= self.graph_dead_max:
                return False
        with torch.no_grad():
            if ent is None:  # static inputs: the graphs read their inputs from fixed addresses
                ent = {"sx": torch.empty(x.shape, dtype=x.dtype, device=x.device), "gbufs": []}
                views = [None] * len(A_in)
                for i, j in groups:
                    src = A_in[i]
                    buf = torch.empty((src.shape[0] * (j - i),) + tuple(src.shape[1:]), dtype=src.dtype,
                                      device=src.device)
                    ent["gbufs"].append(buf)
                    views[i:j] = ops.split_rows(buf, j - i)
                ent["views"] = views
                new = True
            else:
                new = False
            s_audio.wait_stream(main)
            s_text.wait_stream(main)
            with torch.cuda.stream(s_text):
                ent["sx"].copy_(x)
            with torch.cuda.stream(s_audio):
                for (i, j), buf in zip(groups, ent["gbufs"]):
                    buf.copy_(ops.group(A_in[i:j]))
            if new:
                self._capture_dead(ent, live, noise, B, s_audio, s_text)
                self._dgraphs[sig] = ent
            with torch.cuda.stream(s_text):
                ent["text_self"].replay()
            with torch.cuda.stream(s_audio):
                ent["audio"].replay()
                ev = torch.cuda.Event()
                ev.record(s_audio)
            with torch.cuda.stream(s_text):
                s_text.wait_event(ev)
                ent["text_cross"].replay()
        if self.keep_dead_out:
            self.dead_out = ent["out"]
        return True

    def _capture_dead(self, ent, live, noise, B, s_audio, s_text):
        """Record the three dead-block graphs of one signature (inputs: ent's static buffers)."""
        sx, views = ent["sx"], ent["views"]
        graphs = [torch.cuda.CUDAGraph() for _ in range(3)]
        # each graph captured on the stream it replays on (per-stream buffers and caches are that stream's)
        with torch.cuda.graph(graphs[0], stream=s_text, capture_error_mode="thread_local"):
            As = [self._dead_text_self(i, sx, noise) for i in range(live)]
        with torch.cuda.graph(graphs[1], stream=s_audio, capture_error_mode="thread_local"):
            KVs = [self._dead_audio(i, views, noise, B)[1] for i in range(live)]
        with torch.cuda.graph(graphs[2], stream=s_text, capture_error_mode="thread_local"):
            out = [self._dead_text_cross(i, As[i], KVs[i], noise)[-1] for i in range(live)][-1]
        for s in (s_audio, s_text):
            gemm_mod.forget_stream(s.cuda_stream)
        ent.update(text_self=graphs[0], audio=graphs[1], text_cross=graphs[2], out=out,
                   # read across graphs: the text self calls' outputs and the audio side's k / v (each lives in
                   # its producer graph's pool, held here)
                   cross=(As, KVs),
                   # made outside the capture, read by the graphs, droppable by a cache: rotary tables (replaced
                   # when a longer sequence grows them) and the bulk bf16 arena
                   refs=(tuple(ops._ROT_TABLES.values()), gemm_mod.plan_refs()))

    def reset_dead_graphs(self):
        """Drop the captured dead-block graphs (after changing a switch the signature does not cover, e.g. the
        C-side kernel variants of asrx_set_gemm_variant)."""
        self.join_dead_blocks()
        torch.cuda.synchronize()
        self._dgraphs.clear()
        self._dseen.clear()

    def _side_streams(self, device):
        if self._side is None or self._side[0].device != device:
            self._side = (torch.cuda.Stream(device=device), torch.cuda.Stream(device=device))
        return self._side

    def _dead_text_self(self, i, x, noise):
        return ops.fork(self.block[i].call(x, noise, f"b{i}.ta", 0, masked=True))

    def _dead_audio(self, i, A_in, noise, B):
        blk = self.block[i]
        A = self._audio(blk, A_in, noise, f"b{i}.audio", B, "call")
        return A, self._audio(blk, A, noise, f"b{i}.xa", B, "xa")

    def _dead_text_cross(self, i, a, KV, noise):
        blk = self.block[i]
        b_ = ops.fork(blk.call(a, noise, f"b{i}.tb", 0, kv=KV[0]))
        c_ = ops.fork(blk.call(b_, noise, f"b{i}.tc", 0, kv=KV[1]))
        d = ops.fork(blk.call(c_, noise, f"b{i}.td", 0, kv=KV[2]))
        e = ops.add(a, b_, c_)
        kve = blk.xa_side(e, noise, f"b{i}.tg.xa", 0)
        return b_, c_, d, e, kve, blk.call(d, noise, f"b{i}.tg", 0, kv=kve)

    def _dead_block(self, i, x, A_in, noise, B, s_audio, s_text, keep=None):
        """Block i < L-1 without autograd state (model.py:617-626; its output is discarded): the audio side
        on s_audio (None: the current stream), the text side on s_text (None: the current stream) -- the
        text self call first, the cross calls after the audio side's k / v (event).  Returns the block's last
        output."""
        cur = contextlib.nullcontext
        with torch.cuda.stream(s_text) if s_text is not None else cur():
            a = self._dead_text_self(i, x, noise)
        with torch.cuda.stream(s_audio) if s_audio is not None else cur():
            A, KV = self._dead_audio(i, A_in, noise, B)
            ev = None
            if s_text is not None:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
        if keep is not None:
            keep.append(KV)
        with torch.cuda.stream(s_text) if s_text is not None else cur():
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            rest = self._dead_text_cross(i, a, KV, noise)
        # tensors made on one stream and read on another stay referenced until the join
        if keep is not None:
            keep.append((A, KV, a) + rest)
        elif self._hold is not None:
            self._hold.append((A, KV, a) + rest)
        return rest[-1]

    def join_dead_blocks(self):
        """Join the side streams of the concurrent dead blocks into the current stream (idempotent)."""
        p, self._pending = self._pending, None
        if p is not None:
            s_audio, s_text, _, main = p  # the stream the forward (and so its backward) was issued on
            main.wait_stream(s_audio)
            main.wait_stream(s_text)
        self._hold = []

    # ---- decoding (Model.generate): the y-independent audio side of the only live block, once
    def audio_cache(self, xa, noise: NoiseCtx, B: int):
        """The last block's audio self-calls i(xa['a'|'b'|'c']) and their cross-attention k/v
        (model.py:619-622): they do not depend on the text, so generate computes them once.  Earlier
        blocks are dead in processor.forward (each restarts from the embeddings and only the last
        block's d / g reach the output), so they are not run at all when decoding."""
        i = len(self.block) - 1
        blk = self.block[i]
        A = self._audio(blk, [xa["a"], xa["b"], xa["c"]], noise, f"b{i}.audio", B, "call")
        return self._audio(blk, A, noise, f"b{i}.xa", B, "xa")

    def decode_logits(self, x, kv, noise: NoiseCtx):
        """processor.forward(x, xa, seq=True) (model.py:624-629) from an audio_cache: the last
        block's text-side calls a, b, c, d, g and the tied logits."""
        B, T = x.shape
        i = len(self.block) - 1
        blk = self.block[i]
        h = ops.add_rows(ops.Embedding.apply(x, self.token.weight), self.position)
        a = blk.call(h, noise, f"b{i}.ta", 0, masked=True)
        b_ = blk.call(a, noise, f"b{i}.tb", 0, kv=kv[0])
        c_ = blk.call(b_, noise, f"b{i}.tc", 0, kv=kv[1])
        d = blk.call(c_, noise, f"b{i}.td", 0, kv=kv[2])
        e = ops.add(a, b_, c_)
        g = blk.call(d, noise, f"b{i}.tg", 0, kv=blk.xa_side(e, noise, f"b{i}.tg.xa", 0))
        out = self.ln.run(g.contiguous(), noise, "final.ln", 0, T, out_bf16=True)
        return ops.linear(out, self.token.weight)

    @staticmethod
    def _audio(blk, streams, noise, site, B, kind):
        """Run blk.call / blk.xa_side on the 3 audio streams, batching streams of equal length."""
        out = [None, None, None]
        i = 0
        while i < 3:
            j = i + 1
            while j < 3 and streams[j].shape[1] == streams[i].shape[1]:
                j += 1
            x = ops.group(streams[i:j])  # the batched tensor itself when the streams are its views
            if kind == "call":
                y = blk.call(x, noise, site, i * B)
                out[i:j] = ops.split_rows(y, j - i)
            else:
                k, v = blk.xa_side(x, noise, site, i * B)
                for s, kk, vv in zip(range(i, j), ops.split_rows(k, j - i), ops.split_rows(v, j - i)):
                    out[s] = (kk, vv)
            i = j
        return out


def stream_grouping(lengths):
    """Group id of each audio stream: consecutive streams of equal length share one batched pass
    (AudioEncoder.encode, processor._audio), e.g. (0, 0, 1) for pitch and spectrogram at 3001 frames
    and the waveform feature at 3000."""
    out, gid = [], 0
    for i, n in enumerate(lengths):
        if i and n != lengths[i - 1]:
            gid += 1
        out.append(gid)
    return tuple(out)


class Model(nn.Module):
    """model.py:631-701."""

    def __init__(self, param: Dimensions):
        super().__init__()
        hd = param.dims // param.head if param.head > 0 else 0
        if param.head <= 0 or param.dims % param.head or hd not in (64, 128) or param.dims % 64:
            raise ValueError(f"Dimensions(dims={param.dims}, head={param.head}): head dim {hd} unsupported; the "
                             "attention kernels take head dims 64 and 128 (dims a multiple of 64)")
        self.param = param
        self.processor = processor(tokens=param.tokens, mels=param.mels, dims=param.dims, head=param.head,
                                   layer=param.layer, act=param.act, n_type=param.n_type)
        self.enc = AudioEncoder(param.mels, param.dims, param.head, param.layer, param.act, param.n_type,
                                norm=False, enc=False)
        self.layer = sum(1 for name, _ in self.named_modules() if name != "")
        self.noise_seed = 0
        self.noise_step = 0
        # perf mode: the tied logits and the cross entropy run fused (ops.LogitsCE: logits stored bf16,
        # the loss from the GEMM's per-tile statistics); False: logits GEMM then ops.CrossEntropy
        self.fused_ce = True
        # opt-in: the fused path returns the logits stored bf16 (half the logits bytes); default fp32 like
        # the reference (model.py:629 .float())
        self.bf16_logits = False

    def grad_reachable(self):
        """The parameters a training step can give a gradient (asrx.dist.GradSync gives each a bucket
        slot from step 1, zero-filled when a step leaves it without one): all but blocks 0..L-2 (dead:
        they restart from the embeddings and never reach the output, model.py:617-628) and the modules the
        reference constructs but never calls (attention.c, rotary.lin, the router -- applied as the
        identity it is --, AdaptiveSpan.span_scale, processor.pitch_tokens)."""
        L = len(self.processor.block)
        dead = tuple(f"processor.block.{i}." for i in range(L - 1))
        unused = (".attn.c.", ".rot.lin.", ".router.", ".shared_head.span_scale", "processor.pitch_tokens.")
        return [p for n, p in self.named_parameters()
                if p.requires_grad and not n.startswith(dead) and not any(u in n for u in unused)]

    def set_noise(self, seed: int, step: int):
        self.noise_seed, self.noise_step = int(seed), int(step)

    def forward(self, labels=None, text_ids=None, spectrogram=None, pitch=None, waveform=None, pitch_tokens=None):
        if pitch_tokens is not None:
            raise NotImplementedError("pitch_tokens: the reference's pitch-token branch calls an undefined "
                                      "quantize_pitch (model.py:609); out of scope (SURVEY.md §2 #4)")
        first = next((t for t in (pitch, spectrogram, waveform) if t is not None), None)
        if first is None or text_ids is None:
            raise ValueError("forward needs text_ids and at least one of pitch/spectrogram/waveform")

        def aborc(a, b, c):  # essentials.py:25
            return a if a is not None else (b if b is not None else c)

        streams = [aborc(pitch, spectrogram, waveform), aborc(spectrogram, pitch, waveform),
                   aborc(waveform, pitch, spectrogram)]
        # no .contiguous(): the stems read a (B, 128, F) spectrogram through its (B, F, 128) layout
        streams = [s.to(torch.float32) for s in streams]
        B = first.shape[0]
        # how this step is batched decides how many gradient contributions each shared weight gets
        # (runs of consecutive equal-length streams share one pass): asrx.dist.GradSync keys its event
        # plans on that grouping -- not on the raw lengths, which vary from batch to batch
        self.grad_signature = (self.training, stream_grouping([s.shape[-1] for s in streams]))
        gemm_mod.clear_weight_cache(self)
        noise = NoiseCtx(self.noise_seed, self.noise_step, self.training)
        if self.training:
            self.noise_step += 1
        enc = self.enc.encode(streams, noise, B)
        xa = {"a": enc[0], "b": enc[1], "c": enc[2]}
        loss = None
        if labels is not None and self.fused_ce:
            h = self.processor(text_ids, xa, noise, seq=False, features=True)
            if ops.logits_ce_ok(h, self.processor.token.weight):
                logits, loss = ops.logits_ce(h, self.processor.token.weight, labels, self.bf16_logits)
            else:
                logits = ops.linear(h, self.processor.token.weight)
        else:
            logits = self.processor(text_ids, xa, noise, seq=False)
        if labels is not None and loss is None:
            loss = ops.CrossEntropy.apply(logits, labels)
        self._end_step_after(logits, loss)
        return {"logits": logits, "loss": loss}

    def _end_step(self):
        """End of a step: join the dead blocks' side streams, drop the per-step weight copies."""
        self.processor.join_dead_blocks()
        gemm_mod.end_step()

    def end_step(self):
        """End the current step explicitly.  A training step normally ends by itself at the end of the
        backward that follows forward (_end_step_after); a forward run with grad enabled and NO backward
        after it (validation under enable_grad, a step skipped on a NaN loss) otherwise keeps its side-stream
        work and the per-step weight / derived caches (keyed by parameter address) alive until the next
        forward or generate.  Call this before touching parameters directly (an optimizer step, a
        load_state_dict) or before direct asrx.ops calls in such a window.  Idempotent."""
        self._end_step()

    def _end_step_after(self, *outs):
        """The step ends with the backward that follows this forward (an autograd final callback queued
        by a hook on the outputs): the dead blocks on side streams (processor.concurrent_dead_blocks)
        overlap the live block's backward too and are joined before any optimizer step, and the
        per-step weight copies live until then.  Without a backward to come, the step ends now."""
        outs = [t for t in outs if t is not None and t.requires_grad]
        if not (torch.is_grad_enabled() and outs):
            self._end_step()
            return

        def hook(g):
            torch.autograd.Variable._execution_engine.queue_callback(self._end_step)
            return g

        for t in outs:
            t.register_hook(hook)

    @torch.no_grad()
    def generate(self, spectrogram=None, pitch=None, waveform=None, pitch_tokens=None, max_new_tokens=150):
        """Greedy decoding, model.py:674-701: the encoder once, then per new token the processor with
        seq=True on the tokens so far (BOS = 1 first), argmax of the last position, stop when every
        sequence emitted EOS = 2.  Returns LongTensor (B, <= 1 + max_new_tokens).

        The text side is recomputed over the whole prefix each step, as in the reference: its
        self-attention is causal only in call a (calls b, c, d, g attend over the whole text) and
        MSheath pools over positions, so earlier positions change as the text grows and a
        text-side KV cache would change the result.  What is y-independent is cached: the audio
        self-calls and the cross-attention k/v of the live block (processor.audio_cache).  The
        gumbel noise is the model's keyed noise at one (seed, step), the same for every decoding
        step (the reference draws fresh noise per call: its decoding is not reproducible)."""
        if pitch_tokens is not None:
            raise NotImplementedError("pitch_tokens: see Model.forward")
        self.eval()
        first = next((t for t in (pitch, spectrogram, waveform) if t is not None), None)
        if first is None:
            raise ValueError("generate needs at least one of pitch/spectrogram/waveform")

        def aborc(a, b, c):
            return a if a is not None else (b if b is not None else c)

        streams = [aborc(pitch, spectrogram, waveform), aborc(spectrogram, pitch, waveform),
                   aborc(waveform, pitch, spectrogram)]
        streams = [s.to(torch.float32).contiguous() for s in streams]
        B = first.shape[0]
        gemm_mod.clear_weight_cache(self)
        noise = NoiseCtx(self.noise_seed, self.noise_step, False)
        enc = self.enc.encode(streams, noise, B)
        kv = self.processor.audio_cache({"a": enc[0], "b": enc[1], "c": enc[2]}, noise, B)
        y = torch.ones(B, 1, dtype=torch.long, device=first.device)
        for _ in range(max_new_tokens):
            logits = self.processor.decode_logits(y, kv, noise)
            nxt = torch.argmax(logits[:, -1, :], dim=-1, keepdim=True)
            y = torch.cat((y, nxt), dim=1)
            if bool((nxt == 2).all()):
                break
        gemm_mod.end_step()
        return y
