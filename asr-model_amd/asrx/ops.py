"""Autograd functions over the HIP C-ABI.  Forward and backward of every function run asrx kernels
(csrc/*.hip); PyTorch supplies memory, streams and the autograd tape only.

Activations are contiguous device tensors, float32 -- or bfloat16 where an activation's only consumers
are GEMM / attention operands and the perf mode stores it that way (asrx.prec.bf16_storage: the
consumers round to bf16 anyway); "rows" means the flattened leading dims.
"""
from __future__ import annotations

import ctypes
import math
import weakref

import torch

from . import decisions
from . import gemm as G
from . import lib, prec, probe

_E = torch.empty
_S = lib.stream
_P = lib.ptr


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _rows(t):
    return t.numel() // t.shape[-1]


def _zeros_like(t):
    return torch.zeros_like(t)


ACT = G.ACT

# =============================================================================== parameter gradients
# Kernels that produce a leaf parameter's gradient accumulate it straight into p.grad (GEMM beta = 1,
# atomic reductions) instead of returning it to autograd.  A parameter of this model is used 10-50
# times per step (every residual call re-uses its block's weights, AbbyNormal's router runs ~6 times
# per call); returned gradients cost a zero-filled buffer per use plus one autograd sum launch per
# extra use (~3000 small launches per tiny-config step).  `.backward()` semantics are unchanged (p.grad
# holds the sum); torch.autograd.grad(..., inputs=params) needs DIRECT = False.  Every contribution
# that lands is announced to GRAD_LISTENERS (asrx.dist.GradSync counts them to start a bucket's
# all-reduce as soon as the bucket is complete).
DIRECT = True
GRAD_LISTENERS: list = []


def _direct(ctx, i, p):
    """Forward-time decision for input i: True when p's gradient goes straight into p.grad."""
    return DIRECT and p is not None and ctx.needs_input_grad[i] and p.is_leaf


def _gbuf(p, direct):
    """Accumulation target for p's gradient: p.grad (created zeroed on first use) when direct."""
    if not direct:
        return torch.zeros_like(p)
    g = p.grad
    if g is None:
        g = torch.zeros_like(p)
        p.grad = g
    return g


def _gret(p, g, direct):
    """What backward returns for p: None once g (== p.grad) holds the contribution."""
    if not direct:
        return g
    for ref in list(GRAD_LISTENERS):
        fn = ref() if isinstance(ref, weakref.WeakMethod) else ref
        if fn is None:
            GRAD_LISTENERS.remove(ref)
        else:
            fn(p)
    return None

# =============================================================================== multi-consumer activations
# An activation read by several ops gets one gradient per consumer, which autograd sums with stock
# add kernels.  fork(x) instead hands the consumers a GradSink: ops that support it (AbbyNormal,
# Linear, rotary's |src|) accumulate x's gradient straight into the sink's buffer (the first writes,
# later ones add: beta = 1 GEMMs, accumulate-mode row kernels) and return None to autograd;
# ForkFn.backward, which autograd runs after every consumer, returns the buffer (plus, in one asrx
# launch, the gradient of any consumer that did not use the sink).


class GradSink:
    __slots__ = ("buf",)

    def __init__(self):
        self.buf = None

    def target(self, like):
        """(buffer, acc): the first contributor writes its gradient (acc = 0), later ones add."""
        if self.buf is None:
            self.buf = _E(like.shape, device=like.device)
            return self.buf, 0
        return self.buf, 1


class PartSink:
    """The sink of one part (rows [i B, (i+1) B)) of a stream group whose own sink is `parent` (a split
    bf16-stored group, e.g. the cross-attention k / v of equal-length audio streams): contributions land in
    the slice of the parent's buffer, which is allocated zero-filled so every contributor adds."""
    __slots__ = ("parent", "i", "n", "shape")

    def __init__(self, parent, i, n, shape):
        self.parent, self.i, self.n, self.shape = parent, i, n, shape

    def target(self, like):
        if self.parent.buf is None:
            self.parent.buf = torch.zeros(self.shape, device=like.device)
        B = self.shape[0] // self.n
        return self.parent.buf[self.i * B:(self.i + 1) * B].view(like.shape), 1


class ForkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, sink):
        ctx.set_materialize_grads(False)
        ctx.sink = sink
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        sink, ctx.sink = ctx.sink, None
        return grad_in(g, sink), None


def fork(x):
    """x for several consumers whose gradients should meet in one buffer (see above)."""
    if not (torch.is_grad_enabled() and x.requires_grad) or getattr(x, "_asrx_sink", None) is not None:
        return x
    sink = GradSink()
    y = ForkFn.apply(x, sink)
    y._asrx_sink = sink
    return y


def sink_of(x):
    return getattr(x, "_asrx_sink", None)


# =============================================================================== bf16-stored outputs
# A Function whose output is stored bf16 (asrx.prec.bf16_storage) must not receive its gradient through
# autograd: the engine casts every gradient to the dtype of the tensor it belongs to, so it would arrive
# rounded to bf16 (and the kernels take fp32 gradients).  Such an output carries a GradSink instead:
# its consumers (Linear, KVProj, TGate, attention) accumulate their exact fp32 input gradient into the
# sink and return None, and the producer's backward reads the sink (plus, converted, whatever autograd
# delivered from a consumer without sink support).


def out_sink(y, sink):
    """Attach `sink` to the producer's output y (a bf16-stored activation) and return y."""
    if sink is not None and y.requires_grad:
        y._asrx_sink = sink
    return y


def new_sink(out_bf16: bool):
    """A sink for a producer about to store its output bf16 (None when no backward will run)."""
    return GradSink() if (out_bf16 and torch.is_grad_enabled() and prec.bf16_storage()) else None


def grad_in(g, sink):
    """The full fp32 gradient of an output: the sink's buffer (sink-capable consumers) plus the
    autograd-delivered part (None, fp32 or bf16)."""
    buf = None
    if sink is not None:
        buf, sink.buf = sink.buf, None
    if g is not None:
        g = g.float() if g.dtype != torch.float32 else g
        g = _c(g)
    if buf is None:
        return g
    if g is not None:
        lib.call("asrx_lincomb", _P(buf), _P(g), None, 1.0, 1.0, 0.0, _P(buf), buf.numel(), _S())
    return buf


def _f32(g):
    """An incoming gradient as fp32 (autograd delivers bf16 for a bf16 tensor's gradient)."""
    if g is None:
        return None
    return _c(g.float() if g.dtype != torch.float32 else g)


class SplitRows(torch.autograd.Function):
    """A (n B, ...) stream group as n (B, ...) views (equal-length audio streams share one batched
    pass); the backward joins the views' gradients in one kernel instead of autograd's zero-filled
    full-size buffer per view plus an add."""

    @staticmethod
    def forward(ctx, x, n):
        ctx.set_materialize_grads(False)
        ctx.n = n
        ctx.shape = x.shape
        B = x.shape[0] // n
        return tuple(x[i * B:(i + 1) * B] for i in range(n))

    @staticmethod
    def backward(ctx, *gs):
        n = ctx.n
        gs = [_f32(g) for g in gs]  # views of a bf16-stored group get bf16 gradients from autograd
        if all(g is None for g in gs):
            return None, None
        out = _E(ctx.shape, device=next(g for g in gs if g is not None).device)
        per = out.numel() // n
        if all(g is not None for g in gs) and n in (2, 3):
            gs = [_c(g) for g in gs]
            lib.call("asrx_cat3", _P(gs[0]), _P(gs[1]), _P(gs[2]) if n == 3 else None, per, _P(out), _S())
            return out, None
        of = out.view(n, per)
        for i, g in enumerate(gs):
            if g is None:
                lib.call("asrx_zero", _P(of[i]), per * 4, _S())
            else:
                lib.call("asrx_lincomb", _P(_c(g)), None, None, 1.0, 0.0, 0.0, _P(of[i]), per, _S())
        return out, None


def split_rows(x, n):
    """n views of a stream group, tagged so that group(...) can use the group tensor again."""
    if n == 1:
        return [x]
    parts = SplitRows.apply(x, n) if (torch.is_grad_enabled() and x.requires_grad) else \
        tuple(x[i * (x.shape[0] // n):(i + 1) * (x.shape[0] // n)] for i in range(n))
    sk = sink_of(x)
    for i, t in enumerate(parts):
        t._asrx_group = (x, i, n)
        if sk is not None and t.requires_grad:  # consumers of a part add into its slice of x's sink
            t._asrx_sink = PartSink(sk, i, n, tuple(x.shape))
    return list(parts)


def group(parts):
    """The batched tensor of consecutive stream views: the group they were split from when they are
    exactly its parts in order, else one concatenation."""
    if len(parts) == 1:
        return parts[0]
    g = getattr(parts[0], "_asrx_group", None)
    if g is not None and g[2] == len(parts) and all(
            getattr(t, "_asrx_group", (None, -1))[0] is g[0] and t._asrx_group[1] == i for i, t in enumerate(parts)):
        return g[0]
    return torch.cat(parts, 0)


# =============================================================================== Linear (GEMM)


class Linear(torch.autograd.Function):
    """y = act(x W^T + b) on MFMA (nn.Linear / 1x1 Conv1d)."""

    @staticmethod
    def forward(ctx, x, W, b, act="none", grad=True, sink=None, out_bf16=False, osink=None):
        x = _c(x)
        ctx.sink = sink
        ctx.osink = osink
        ctx.set_materialize_grads(False)
        # the pre-activation is kept only for a backward that will run (none in the reference's dead
        # blocks, eval or decoding: an N-wide fp32 write saved per call)
        # perf mode: the backward's GEMM recomputes the pre-activation (gemm_wn_gact) instead of reading it
        ctx.recompute = grad and G.can_recompute_act(x, W, act)
        z = _E(*x.shape[:-1], W.shape[0], device=x.device) if act != "none" and grad and not ctx.recompute else None
        y = G.linear_fwd(x, W.view(W.shape[0], -1), b, act=act, preact=z,  # (N, K, 1): a 1x1 Conv1d weight
                         out_bf16=out_bf16 and prec.bf16_storage())
        ctx.act = act
        ctx.has_b = b is not None
        if grad:
            ctx.dW, ctx.db = _direct(ctx, 1, W), _direct(ctx, 2, b)
            # the bias itself (not only its gradient target) when the backward recomputes z = x W^T + b
            ctx.save_for_backward(x, W, z, b if (ctx.db or ctx.recompute) else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W3, z, b = ctx.saved_tensors
        W = W3.view(W3.shape[0], -1)
        ctx.bias_t = b if ctx.has_b else None
        gy = grad_in(gy, ctx.osink)
        if gy is None:
            return None, None, None, None, None, None, None, None
        db_done = None
        N = gy.shape[-1]
        if ctx.recompute:
            gz = _E(gy.shape, dtype=torch.bfloat16, device=gy.device)
            if ctx.has_b and ctx.needs_input_grad[2]:
                db_done = _gbuf(b, True) if ctx.db else torch.zeros(N, device=gy.device)
            G.linear_gact(x, W, ctx.bias_t, _c(gy), gz, ctx.act, db=db_done)
        elif ctx.act in ("gelu", "silu", "sigmoid") and prec.get() == prec.PREC_BF16 and N % 8 == 0 and G.use_wide(N):
            # perf mode: act' applied, gz stored bf16 for the two GEMMs and the bias gradient summed in
            # the same pass (no fp32 gz round trip, no separate column-sum pass)
            gz = _E(gy.shape, dtype=torch.bfloat16, device=gy.device)
            if ctx.has_b and ctx.needs_input_grad[2]:
                db_done = _gbuf(b, True) if ctx.db else torch.zeros(N, device=gy.device)
            lib.call("asrx_act_bwd_bias", _P(_c(gy)), _P(z), _P(gz), _P(db_done), _rows(gy), N, ACT[ctx.act], _S())
        elif ctx.act != "none":
            gz = _E(gy.shape, device=gy.device)
            lib.call("asrx_act_bwd", _P(gy), _P(z), _P(gz), gy.numel(), ACT[ctx.act], _S())
        else:
            gz = gy
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(x)
                G.linear_dgrad(gz, W, out=buf, beta=float(acc))
            else:
                dx = G.linear_dgrad(gz, W)
        dW = db = None
        gb = None
        if db_done is None and ctx.has_b and ctx.needs_input_grad[2]:
            gb = _gbuf(b, True) if ctx.db else torch.zeros(N, device=gy.device)
        if ctx.needs_input_grad[1]:
            gW = _gbuf(W3, ctx.dW)
            G.linear_wgrad(gz, x, out=gW.view(W.shape), accumulate=True, db=gb)  # bias gradient in the same pass
            dW = _gret(W3, gW, ctx.dW)
            if gb is not None:
                db_done, gb = gb, None
        if db_done is not None:
            db = _gret(b, db_done, ctx.db)
        elif gb is not None:
            db = _gret(b, colsum(gz, out=gb), ctx.db)
        return dx, dW, db, None, None, None, None, None


def _grad_needed(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def linear(x, W, b=None, act="none", out_bf16=False):
    """nn.Linear (+ act) on MFMA; out_bf16: the output only feeds GEMM operands (stored bf16 in perf mode)."""
    grad = _grad_needed(x, W, b)
    osink = new_sink(out_bf16) if grad else None
    return out_sink(Linear.apply(x, W, b, act, grad, sink_of(x), out_bf16, osink), osink)


class LinearRes(torch.autograd.Function):
    """y = r + x W^T + b: the residual add around an out projection (model.py:578-580 x = x +
    attn(...)) in the GEMM's epilogue (perf mode) -- no separate add pass; backward: r's gradient is y's
    (passed through), x / W / b as Linear."""

    @staticmethod
    def forward(ctx, r, x, W, b, sink=None):
        x, r = _c(x), _c(r)
        ctx.sink = sink
        ctx.set_materialize_grads(False)
        x2 = x.view(-1, x.shape[-1])
        if G.is_bf16(x2):
            raise RuntimeError("LinearRes: the residual epilogue takes an fp32 x (use ops.linear_residual)")
        M, K = x2.shape
        N = W.shape[0]
        y = _E(r.shape, device=r.device)
        Wb = G.weight_bf16(W)
        nj = G._nj(M, N)
        e0 = probe.begin("gemm")
        lib.call("asrx_gemm_wn_res", _P(x2), K, _P(Wb), Wb.stride(0), _P(y), N, _P(b), _P(r), N, M, N, K, nj, _S())
        probe.end("gemm", e0, 2.0 * M * N * K, ("wn", M, N, K, nj, 0, "none", False, True, 0, 0, -1))
        ctx.dW, ctx.db = _direct(ctx, 2, W), _direct(ctx, 3, b)
        ctx.save_for_backward(x, W, b if ctx.db else None)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, b = ctx.saved_tensors
        if gy is None:
            return None, None, None, None, None
        gy = _f32(gy)
        dx = None
        if ctx.needs_input_grad[1]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(x)
                G.linear_dgrad(gy, W, out=buf, beta=float(acc))
            else:
                dx = G.linear_dgrad(gy, W)
        dW = db = None
        gb = None
        if ctx.has_b and ctx.needs_input_grad[3]:
            gb = _gbuf(b, True) if ctx.db else torch.zeros(W.shape[0], device=gy.device)
        if ctx.needs_input_grad[2]:
            gW = _gbuf(W, ctx.dW)
            G.linear_wgrad(gy, x, out=gW, accumulate=True, db=gb)  # bias gradient in the same pass
            dW = _gret(W, gW, ctx.dW)
        elif gb is not None:
            colsum(gy, out=gb)
        if gb is not None:
            db = _gret(b, gb, ctx.db)
        return gy if ctx.needs_input_grad[0] else None, dx, dW, db, None


def linear_residual(r, x, W, b=None):
    """r + nn.Linear(x): fused in perf mode (LinearRes), else add(r, linear(x))."""
    N = W.shape[0]
    K = x.shape[-1]
    M = x.numel() // max(K, 1)
    if (prec.get() == prec.PREC_BF16 and G.use_wide(K) and N % 4 == 0 and r.dtype == torch.float32
            and x.dtype == torch.float32 and r.shape[-1] == N and x.is_cuda and G._nj(M, N) in (1, 3)):
        return LinearRes.apply(r, x, W, b, sink_of(x))
    return add(r, linear(x, W, b))


class KVProjFn(torch.autograd.Function):
    """k, v = Linear(D, 2D) of the same normed source, split '(kv h d)' (model.py:261): two GEMMs on
    the weight's row blocks (no copies), backward with both input gradients meeting in one buffer
    (beta = 1) and the weight / bias gradients written into the blocks of p.grad."""

    @staticmethod
    def forward(ctx, x, W, b, sink, v_bf16=False, vsink=None, src=None, rot=None, grad=False):
        """rot: (freqs, hd, scale, src sink, ||src|| or None) -- k leaves the GEMM rotated (asrx_gemm_wn_rot,
        model.py:304's rotary of k on the kv source src), its unrotated product kept for the backward."""
        x = _c(x)
        D = W.shape[0] // 2
        ctx.rot = rot is not None
        if rot is not None:
            freqs, hd, scale, ctx.src_sink, m = rot
            src = _c(src)
            L = x.shape[1]
            if m is None:
                m = _E(_rows(src), device=x.device)
                lib.call("asrx_rownorm", _P(src), _P(m), _rows(src), src.shape[-1], _S())
            tab = rotary_table(freqs, L, hd)
            kz = _E(*x.shape[:-1], D, device=x.device) if grad else None
            k = G.linear_rot_fwd(x, W[:D], b[:D], m, tab, L, hd, scale, preact=kz)
            ctx.hd, ctx.scale = hd, scale
            # (kz, src, m, freqs, tab) through save_for_backward like LinearRotFn: autograd's version check
            # then catches an in-place change of src or its row norm between forward and backward
            rsaved = (kz, src, m, freqs, tab) if grad else (None,) * 5
        else:
            k = G.linear_fwd(x, W[:D], b[:D])
            rsaved = (None,) * 5
        v = G.linear_fwd(x, W[D:], b[D:], out_bf16=v_bf16)  # v only feeds attention
        ctx.vsink = vsink
        ctx.set_materialize_grads(False)
        ctx.sink = sink
        ctx.dW, ctx.db = _direct(ctx, 1, W), _direct(ctx, 2, b)
        ctx.save_for_backward(x, W, b, *rsaved)
        return k, v

    @staticmethod
    def backward(ctx, dk, dv):
        x, W, b, *rsaved = ctx.saved_tensors
        D = W.shape[0] // 2
        dk = _f32(dk)
        dv = grad_in(dv, ctx.vsink)
        dsrc = None
        if ctx.rot and dk is not None and rsaved[1] is not None:
            dk, dsrc = _rotary_bwd(ctx, dk, *rsaved, ctx.needs_input_grad[6], ctx.src_sink)
        if dk is not None:
            dk = dk.reshape(*x.shape[:-1], D)
        if dv is not None:
            dv = dv.reshape(*x.shape[:-1], D)  # a sink buffer may hold the (B, L, H, hd) view's shape
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(x)
            else:
                buf, acc = _E(x.shape, device=x.device), 0
            for gpart, Wp in ((dk, W[:D]), (dv, W[D:])):
                if gpart is not None:
                    G.linear_dgrad(gpart, Wp, out=buf, beta=float(acc))
                    acc = 1
            if acc == 0:
                lib.call("asrx_zero", _P(buf), buf.numel() * 4, _S())
            dx = None if ctx.sink is not None else buf
        dWf = dbf = None
        if ctx.needs_input_grad[1]:
            gW = _gbuf(W, ctx.dW)
            gb = _gbuf(b, ctx.db) if ctx.needs_input_grad[2] else None
            for i, gpart in enumerate((dk, dv)):
                if gpart is not None:
                    G.linear_wgrad(gpart, x, out=gW[i * D:(i + 1) * D], accumulate=True,
                                   db=None if gb is None else gb[i * D:(i + 1) * D])
            dWf = _gret(W, gW, ctx.dW)
            if gb is not None:
                dbf = _gret(b, gb, ctx.db)
        elif ctx.needs_input_grad[2]:
            gb = _gbuf(b, ctx.db)
            for i, gpart in enumerate((dk, dv)):
                if gpart is not None:
                    colsum(gpart.view(-1, D), out=gb[i * D:(i + 1) * D])
            dbf = _gret(b, gb, ctx.db)
        return dx, dWf, dbf, None, None, None, dsrc, None, None


def kv_proj(x, W, b):
    vb = prec.attn_bf16_io()
    vsink = new_sink(vb) if _grad_needed(x, W, b) else None
    k, v = KVProjFn.apply(x, W, b, sink_of(x), vb, vsink)
    return k, out_sink(v, vsink)


def _rot_fusable(x, N, hd):
    """The rotary can ride in the projection GEMM's epilogue (asrx_gemm_wn_rot): perf mode, a (B, L, K) CUDA
    input, and a tile width the rotary instantiations cover (nj 1 or 3)."""
    K = x.shape[-1]
    return (ROT_FUSED and prec.get() == prec.PREC_BF16 and G.use_wide(K) and x.is_cuda and x.dim() == 3
            and N % 4 == 0 and hd % 4 == 0 and N % hd == 0 and G._nj(_rows(x), N) in (1, 3))


def kv_proj_rotary(x, W, b, src, freqs, hd, scale):
    """(rotary(k, src), v) of kv_proj(x, W, b): the rotary of k fused into its GEMM in perf mode."""
    D = W.shape[0] // 2
    if not _rot_fusable(x, D, hd):
        k, v = kv_proj(x, W, b)
        return rotary(k, src, freqs, hd, scale), v
    vb = prec.attn_bf16_io()
    grad = _grad_needed(x, W, b, src)
    vsink = new_sink(vb) if grad else None
    k, v = KVProjFn.apply(x, W, b, sink_of(x), vb, vsink, src, (freqs, hd, scale, sink_of(src), rownorm_of(src)),
                          grad)
    return k, out_sink(v, vsink)


def colsum(x2, out=None):
    """Column sums of (rows, d), accumulated into `out` when given."""
    d = x2.shape[-1]
    if out is None:
        out = torch.zeros(d, device=x2.device)
    lib.call("asrx_colsum", _P(x2), _P(out), _rows(x2), d, _S())
    return out


class SmallLinear(torch.autograd.Function):
    """y = act(x W^T + b) for <= 4 outputs (row-dot kernel); act in {none, sigmoid}."""

    @staticmethod
    def forward(ctx, x, W, b, act="none"):
        x = _c(x)
        N, K = W.shape
        y = _E(*x.shape[:-1], N, device=x.device)
        lib.call("asrx_small_linear_fwd", _P(x), _P(W), _P(b), _P(y), _rows(x), K, N, ACT[act], _S())
        ctx.act = act
        ctx.has_b = b is not None
        ctx.dW, ctx.db = _direct(ctx, 1, W), _direct(ctx, 2, b)
        ctx.save_for_backward(x, W, y, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y, b = ctx.saved_tensors
        gy = _c(gy)
        N, K = W.shape
        dx = _E(x.shape, device=x.device) if ctx.needs_input_grad[0] else None
        dW = _gbuf(W, ctx.dW)
        db = (_gbuf(b, True) if ctx.db else torch.zeros(N, device=W.device)) if ctx.has_b else None
        lib.call("asrx_small_linear_bwd", _P(gy), _P(y), _P(x), _P(W), _P(dx), _P(dW), _P(db), _rows(x), K, N,
                 ACT[ctx.act], 0.0, _S())
        return dx, _gret(W, dW, ctx.dW), (_gret(b, db, ctx.db) if ctx.has_b else None), None


def small_linear(x, W, b=None, act="none"):
    return SmallLinear.apply(x, W, b, act)


# =============================================================================== AbbyNormal


# The router-epilogue GEMM keeps a whole d-wide row per tile (one 128-row x 384 tile per workgroup): below
# this many rows it runs on too few workgroups (64 at the text side's 8192 rows, 40-48 us per launch), and
# the plain GEMM (128 x 128 tiles, 3x the workgroups) + the row kernel's own SiLU / Linear(d, 3) is faster
ROUTER_FUSED_MIN_ROWS = 32768


class AbbyNormalFn(torch.autograd.Function):
    """essentials.AbbyNormal (essentials.py:155-191): router GEMM on MFMA + fused row kernel."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, L, H, sid_base, key, use_noise, keep, sink=None, out_bf16=False,
                osink=None, tw=None, tb=None, side=None, res=None):
        x = _c(x)
        ctx.has_res = res is not None
        ctx.sink = sink
        ctx.osink = osink
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        rows = _rows(x)
        ob = int(out_bf16 and prec.bf16_storage())
        out = _E(x.shape, device=x.device, dtype=torch.bfloat16 if ob else torch.float32)
        ys = _E(rows, 3, device=x.device)
        idx = _E(rows, dtype=torch.int32, device=x.device)
        # tw / tb: the consuming tgate's cs Linear(d, 3), evaluated on the fp32 output rows in the kernel
        # (a constant for this node: tgate's own backward differentiates it)
        tc = _E(rows, 3, device=x.device) if tw is not None else None
        if side is not None:
            side["tgate_c"] = tc
        cond = None
        if decisions.active():  # record mode 2's per-feature max-vs-avg choices of this call
            cond = torch.zeros(rows, d, dtype=torch.uint8, device=x.device)
            lib.call("asrx_abby_record_cond", _P(cond))
        if res is not None:  # out = res + AbbyNormal(x): the residual add in the same row pass
            res = _c(res)
            if G.use_wide(d) and d <= 384 and rows >= ROUTER_FUSED_MIN_ROWS:
                hpre, logits = G.router_fwd(x.view(rows, d), W1, b1, W2, keep)
            else:
                hpre, logits = G.linear_fwd(x, W1, b1), None
            lib.call("asrx_abby_fwd_res", _P(x), _P(hpre), _P(W2), _P(logits), _P(b2), _P(res), _P(out), _P(ys),
                     _P(idx), rows, d, L, H, sid_base, key & 0xFFFFFFFF, int(use_noise), _S())
        elif side is not None and side.get("want_norm"):  # also ||x[r]|| for rotary's |src|
            if G.use_wide(d) and d <= 384 and rows >= ROUTER_FUSED_MIN_ROWS:
                hpre, logits = G.router_fwd(x.view(rows, d), W1, b1, W2, keep)
            else:
                hpre, logits = G.linear_fwd(x, W1, b1), None
            nrm = _E(rows, device=x.device)
            lib.call("asrx_abby_fwd3", _P(x), _P(hpre), _P(W2), _P(logits), _P(b2), _P(out), ob, _P(ys), _P(idx),
                     rows, d, L, H, sid_base, key & 0xFFFFFFFF, int(use_noise), _P(tw), _P(tb), _P(tc), _P(nrm), _S())
            side["rownorm"] = nrm
        elif G.use_wide(d) and d <= 384 and rows >= ROUTER_FUSED_MIN_ROWS:
            # perf mode: the router's d x d GEMM also applies SiLU and Linear(d, 3) in its epilogue,
            # so h_pre never makes the HBM round trip unless the backward needs it
            hpre, logits = G.router_fwd(x.view(rows, d), W1, b1, W2, keep)
            lib.call("asrx_abby_fwd_logits2", _P(x), _P(logits), _P(b2), _P(out), ob, _P(ys), _P(idx), rows, d, L, H,
                     sid_base, key & 0xFFFFFFFF, int(use_noise), _P(tw), _P(tb), _P(tc), _S())
        else:
            hpre = G.linear_fwd(x, W1, b1)
            lib.call("asrx_abby_fwd2", _P(x), _P(hpre), _P(W2), _P(b2), _P(out), ob, _P(ys), _P(idx), rows, d, L, H,
                     sid_base, key & 0xFFFFFFFF, int(use_noise), _P(tw), _P(tb), _P(tc), _S())
        if cond is not None:
            lib.call("asrx_abby_record_cond", None)
            decisions.abby(key & 0xFFFFFFFF, sid_base, L, H, idx, cond)
        ctx.dp = [_direct(ctx, i, t) for i, t in ((1, W1), (2, b1), (3, W2), (4, b2))]
        ctx.save_for_backward(x, hpre, W1, W2, ys, idx, b1, b2)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, hpre, W1, W2, ys, idx, b1, b2 = ctx.saved_tensors
        gout = grad_in(gout, ctx.osink)
        if gout is None:
            return (None,) * 18
        d = x.shape[-1]
        rows = _rows(x)
        fW1, fb1, fW2, fb2 = ctx.dp
        if ctx.sink is not None:
            dx, acc = ctx.sink.target(x)
        else:
            dx, acc = _E(x.shape, device=x.device), 0
        dh = _E(x.shape, device=x.device)
        dW2, db2 = _gbuf(W2, fW2), _gbuf(b2, fb2)
        lib.call("asrx_abby_bwd2", _P(gout), _P(x), _P(hpre), _P(W2), _P(ys), _P(idx), _P(dx), _P(dh), _P(dW2),
                 _P(db2), rows, d, acc, _S())
        G.linear_dgrad(dh, W1, out=dx, beta=1.0)
        if ctx.sink is not None:
            dx = None
        db1 = _gbuf(b1, fb1)  # bias gradient summed in the weight-gradient pass
        dW1 = G.linear_wgrad(dh, x, out=_gbuf(W1, fW1), accumulate=True, db=db1)
        return (dx, _gret(W1, dW1, fW1), _gret(b1, db1, fb1), _gret(W2, dW2, fW2), _gret(b2, db2, fb2),
                None, None, None, None, None, None, None, None, None, None, None, None,
                gout if ctx.has_res and ctx.needs_input_grad[17] else None)


def abby_normal(mod, x, L, H, sid_base, key, use_noise=True, out_bf16=False, tgate=None, residual=None):
    """AbbyNormal(x); out_bf16: the output only feeds GEMM / attention operands (bf16-stored in perf mode);
    tgate: the consuming tgate module, whose cs Linear(d, 3) the kernel evaluates on the fp32 output (the
    output is then attached to the result for ops.tgate); residual: return residual + AbbyNormal(x),
    the add fused into the kernel (perf mode, H == 1, d >= 128)."""
    if residual is not None and not (prec.get() == prec.PREC_BF16 and H == 1 and x.shape[-1] >= 128
                                     and not out_bf16 and tgate is None and residual.dtype == torch.float32):
        return add(residual, abby_normal(mod, x, L, H, sid_base, key, use_noise, out_bf16, tgate))
    if use_noise:
        _noise_rows_ok(sid_base + _rows(x) // max(L * H, 1), H, L, 3)
    r = mod.mode_router
    keep = torch.is_grad_enabled() and (x.requires_grad or r[0].weight.requires_grad)
    osink = new_sink(out_bf16) if keep else None
    tw = tb = None
    if tgate is not None and H == 1 and x.shape[-1] >= 128:
        tw, tb = tgate.cs[0].weight, tgate.cs[0].bias
    side = {}
    if (getattr(x, "_asrx_want_norm", False) and H == 1 and x.shape[-1] >= 128 and residual is None
            and x.is_cuda and rownorm_of(x) is None):
        side["want_norm"] = True
    y = AbbyNormalFn.apply(x, r[0].weight, r[0].bias, r[2].weight, r[2].bias, L, H, sid_base, key, use_noise,
                           keep, sink_of(x), out_bf16, osink, tw, tb, side, residual)
    if tw is not None:
        y._asrx_tgate_c = (side["tgate_c"], tw)  # tgate's cs logits of these rows, for ops.tgate
    if "rownorm" in side:
        x._asrx_rownorm = (x._version, _S(), side["rownorm"])
    return out_sink(y, osink)


def want_rownorm(x):
    """Ask the AbbyNormal that reads x next to also write ||x[r]|| (rotary's |src|, model.py:201)."""
    x._asrx_want_norm = True
    return x


def rownorm_of(x):
    """||x[r]|| (rows,) left on x by its AbbyNormal (want_rownorm), or None; the tensor's version
    counter guards against an in-place change since, the stream against a read on another stream than
    the one that wrote it (the processor runs blocks on side streams)."""
    c = getattr(x, "_asrx_rownorm", None)
    return c[2] if c is not None and c[0] == x._version and c[1] == _S() else None


# =============================================================================== LayerNorm


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        x = _c(x)
        d = x.shape[-1]
        rows = _rows(x)
        y = _E(x.shape, device=x.device)
        mean = _E(rows, device=x.device)
        rstd = _E(rows, device=x.device)
        lib.call("asrx_layernorm_fwd", _P(x), _P(w), _P(b), _P(y), _P(mean), _P(rstd), rows, d, float(eps), _S())
        ctx.dw, ctx.db = _direct(ctx, 1, w), _direct(ctx, 2, b)
        ctx.save_for_backward(x, w, mean, rstd, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, mean, rstd, b = ctx.saved_tensors
        gy = _c(gy)
        d = x.shape[-1]
        dx = _E(x.shape, device=x.device)
        dw, db = _gbuf(w, ctx.dw), _gbuf(b, ctx.db)
        lib.call("asrx_layernorm_bwd", _P(gy), _P(x), _P(w), _P(mean), _P(rstd), _P(dx), _P(dw), _P(db), _rows(x),
                 d, _S())
        return dx, _gret(w, dw, ctx.dw), _gret(b, db, ctx.db), None


def layer_norm(x, w, b, eps=1e-5):
    return LayerNormFn.apply(x, w, b, eps)


# =============================================================================== attention


def _st3(t):
    """(B, L, H, hd) view -> int64[3] {batch, seq, head} strides."""
    arr = (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2))
    return arr


def _addr(arr):
    return ctypes.cast(arr, ctypes.c_void_p)


class AttentionFn(torch.autograd.Function):
    """SDPA(q, k, v, is_causal) (model.py:307) on (B, L, H, hd) views; scale 1/sqrt(hd).  q / k / v are
    stored fp32 or bf16 (all the same); o is stored bf16 when out_bf16 (it only feeds the out
    projection) -- bf16 storage needs the bf16 flash kernels."""

    @staticmethod
    def forward(ctx, q, k, v, causal, out_bf16=False, sinks=(None, None, None), osink=None, merge=False):
        ctx.set_materialize_grads(False)
        ctx.sinks, ctx.osink = sinks, osink
        B, Lq, H, hd = q.shape
        Lk = k.shape[1]
        ap = prec.attention_prec()
        ib = G.is_bf16(q)
        if not (G.is_bf16(k) == ib and G.is_bf16(v) == ib) or (ib and ap != prec.PREC_BF16):
            q, k, v = q.float(), k.float(), v.float()  # mixed or non-bf16-kernel: fp32 storage
            ib = False
        ob = bool(out_bf16) and ap == prec.PREC_BF16 and prec.bf16_storage()
        o = _E(B, Lq, H, hd, device=q.device, dtype=torch.bfloat16 if ob else torch.float32)
        lse = _E(B, H, Lq, device=q.device)
        sq, sk, sv, so = _st3(q), _st3(k), _st3(v), _st3(o)
        io = int(ib) | (2 * int(ob))
        e0 = probe.begin("attn")
        lib.call("asrx_attn_fwd2", ap, io, _P(q), _addr(sq), _P(k), _addr(sk), _P(v), _addr(sv), _P(o), _addr(so),
                 _P(lse), B, H, Lq, Lk, hd, int(causal), 1.0 / math.sqrt(hd), _S())
        probe.end("attn", e0, 4.0 * B * H * Lq * Lk * hd * (0.5 if causal else 1.0), ("attn", Lq, Lk, io))
        ctx.causal = causal
        ctx.prec = prec.attention_bwd_prec()
        ctx.io = io
        ctx.save_for_backward(q, k, v, o, lse)
        # merge: heads merged '(h d)' (model.py:316), the out projection's input
        return o.view(B, Lq, H * hd) if merge else o

    @staticmethod
    def backward(ctx, go):
        q, k, v, o, lse = ctx.saved_tensors
        go = grad_in(go, ctx.osink)
        if go is None:
            return None, None, None, None, None, None, None, None
        B, Lq, H, hd = q.shape
        go = go.view(B, Lq, H, hd)
        Lk = k.shape[1]
        # an input with a sink (bf16-stored q / k / v): its gradient goes into the sink -- written by the
        # kernel when this is the first contributor, added otherwise
        outs, adds = [], []
        for t, sk in zip((q, k, v), ctx.sinks):
            if sk is not None:
                buf, acc = sk.target(t)
                if acc == 0:
                    outs.append(buf.view(t.shape))
                    adds.append(None)
                    continue
                tmp = _E(t.shape, device=q.device)
                outs.append(tmp)
                adds.append(buf)
            else:
                outs.append(_E(t.shape, device=q.device))
                adds.append(None)
        dq, dk, dv = outs
        delta = _E(B, H, Lq, device=q.device)
        io = ctx.io | (4 * int(G.is_bf16(go)))
        arrs = [_st3(t) for t in (q, k, v, o, go, dq, dk, dv)]
        lib.call("asrx_attn_bwd2", ctx.prec, io, _P(q), _addr(arrs[0]), _P(k), _addr(arrs[1]), _P(v), _addr(arrs[2]),
                 _P(o), _addr(arrs[3]), _P(go), _addr(arrs[4]), _P(lse), _P(delta), _P(dq), _addr(arrs[5]), _P(dk),
                 _addr(arrs[6]), _P(dv), _addr(arrs[7]), B, H, Lq, Lk, hd, int(ctx.causal), 1.0 / math.sqrt(hd),
                 _S())
        res = []
        for g, buf, sk in zip((dq, dk, dv), adds, ctx.sinks):
            if buf is not None:
                lib.call("asrx_lincomb", _P(buf), _P(g), None, 1.0, 1.0, 0.0, _P(buf), buf.numel(), _S())
            res.append(None if sk is not None else g)
        return res[0], res[1], res[2], None, None, None, None, None


def attention(q, k, v, causal, out_bf16=False, merge_heads=False):
    """SDPA (model.py:307) on (B, L, H, hd) -> (B, Lq, H, hd), or (B, Lq, H * hd) with merge_heads;
    out_bf16: the output only feeds the out projection (stored bf16 in perf mode)."""
    grad = _grad_needed(q, k, v)
    osink = new_sink(out_bf16) if grad else None
    sinks = tuple(sink_of(t) for t in (q, k, v)) if grad else (None, None, None)
    return out_sink(AttentionFn.apply(q, k, v, causal, out_bf16, sinks, osink, merge_heads), osink)


# =============================================================================== rotary


class RotaryFn(torch.autograd.Function):
    """rotary.forward (model.py:198-214) fused with the hd^-0.25 scale: x, src (B, L, D)."""

    @staticmethod
    def forward(ctx, x, src, freqs, hd, scale, sink=None, m=None):
        x = _c(x)
        src = _c(src)
        ctx.sink = sink
        B, L, D = x.shape
        if m is None:  # else ||src[r]|| written by src's AbbyNormal (want_rownorm)
            m = _E(B * L, device=x.device)
            lib.call("asrx_rownorm", _P(src), _P(m), B * L, D, _S())
        y = _E(x.shape, device=x.device)
        tab = rotary_table(freqs, L, hd)
        lib.call("asrx_rotary_fwd2", _P(x), _P(m), _P(freqs), _P(tab), _P(y), B * L, L, D, hd, float(scale), _S())
        ctx.hd, ctx.scale = hd, scale
        ctx.save_for_backward(x, src, m, freqs, tab)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, src, m, freqs, tab = ctx.saved_tensors
        gy = _c(gy)
        B, L, D = x.shape
        dx = _E(x.shape, device=x.device)
        dm = _E(B * L, device=x.device)  # written by the kernel
        lib.call("asrx_rotary_bwd2", _P(gy), _P(x), _P(m), _P(freqs), _P(tab), _P(dx), _P(dm), B * L, L, D, ctx.hd,
                 float(ctx.scale), _S())
        dsrc = None
        if ctx.needs_input_grad[1]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(src)
            else:
                buf, acc = _E(src.shape, device=src.device), 0
            lib.call("asrx_rownorm_bwd2", _P(dm), _P(src), _P(m), _P(buf), B * L, D, acc, _S())
            dsrc = None if ctx.sink is not None else buf
        return dx, dsrc, None, None, None, None, None


def _rotary_bwd(ctx, gy, x, src, m, freqs, tab, want_src, src_sink):
    """RotaryFn.backward's arithmetic: -> (dx, dsrc or None); dsrc lands in src_sink when there is one."""
    gy = _c(gy)
    B, L, D = x.shape
    dx = _E(x.shape, device=x.device)
    dm = _E(B * L, device=x.device)  # written by the kernel
    lib.call("asrx_rotary_bwd2", _P(gy), _P(x), _P(m), _P(freqs), _P(tab), _P(dx), _P(dm), B * L, L, D, ctx.hd,
             float(ctx.scale), _S())
    dsrc = None
    if want_src:
        if src_sink is not None:
            buf, acc = src_sink.target(src)
        else:
            buf, acc = _E(src.shape, device=src.device), 0
        lib.call("asrx_rownorm_bwd2", _P(dm), _P(src), _P(m), _P(buf), B * L, src.shape[-1], acc, _S())
        dsrc = None if src_sink is not None else buf
    return dx, dsrc


# perf mode: the q / k projections apply the rotary in their GEMM's epilogue (LinearRotFn, KVProjFn rot);
# False: the projection GEMM then RotaryFn's separate pass (same results, bit for bit)
ROT_FUSED = True


class LinearRotFn(torch.autograd.Function):
    """rotary(Linear(x), src) -- the q projection (model.py:242-245) and its rotary (model.py:198-214, with the
    hd^-0.25 scale of model.py:303) in one GEMM whose epilogue rotates the product before storing it
    (asrx_gemm_wn_rot): the unrotated projection reaches HBM only as the backward's saved input.  Backward:
    RotaryFn's, then Linear's (act none), with the same sinks."""

    @staticmethod
    def forward(ctx, x, W, b, src, freqs, hd, scale, grad=False, sink=None, src_sink=None, m=None):
        x = _c(x)
        src = _c(src)
        ctx.sink, ctx.src_sink = sink, src_sink
        ctx.set_materialize_grads(False)
        L = x.shape[1]
        if m is None:
            m = _E(_rows(src), device=x.device)
            lib.call("asrx_rownorm", _P(src), _P(m), _rows(src), src.shape[-1], _S())
        tab = rotary_table(freqs, L, hd)
        z = _E(*x.shape[:-1], W.shape[0], device=x.device) if grad else None
        y = G.linear_rot_fwd(x, W, b, m, tab, L, hd, scale, preact=z)
        ctx.hd, ctx.scale = hd, scale
        ctx.has_b = b is not None
        if grad:
            ctx.dW, ctx.db = _direct(ctx, 1, W), _direct(ctx, 2, b)
            ctx.save_for_backward(x, W, b, z, src, m, freqs, tab)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, b, z, src, m, freqs, tab = ctx.saved_tensors
        if gy is None:
            return (None,) * 11
        dq, dsrc = _rotary_bwd(ctx, _f32(gy), z, src, m, freqs, tab, ctx.needs_input_grad[3], ctx.src_sink)
        N = W.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(x)
                G.linear_dgrad(dq, W, out=buf, beta=float(acc))
            else:
                dx = G.linear_dgrad(dq, W)
        dW = db = gb = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = _gbuf(b, True) if ctx.db else torch.zeros(N, device=dq.device)
        if ctx.needs_input_grad[1]:
            gW = _gbuf(W, ctx.dW)
            G.linear_wgrad(dq, x, out=gW, accumulate=True, db=gb)  # bias gradient in the same pass
            dW = _gret(W, gW, ctx.dW)
        elif gb is not None:
            colsum(dq.view(-1, N), out=gb)
        if gb is not None:
            db = _gret(b, gb, ctx.db)
        return dx, dW, db, dsrc, None, None, None, None, None, None, None


def linear_rotary(x, W, b, src, freqs, hd, scale):
    """rotary(linear(x, W, b), src, freqs, hd, scale) -- one fused GEMM in perf mode (LinearRotFn)."""
    if not _rot_fusable(x, W.shape[0], hd):
        return rotary(linear(x, W, b), src, freqs, hd, scale)
    grad = _grad_needed(x, W, b, src)
    return LinearRotFn.apply(x, W, b, src, freqs, hd, scale, grad, sink_of(x), sink_of(src), rownorm_of(src))


_ROT_TABLES = {}  # (freqs ptr, hd, device) -> (cap, hd/2, 2) table of positions [0, cap)
_ROT_QUANTUM = 512


def rotary_table(freqs, L, hd):
    """(cos, sin) of position * freqs[j] for positions [0, cap >= L) (asrx_rotary_table).  Row l of the table
    does not depend on the length it was built for, so ONE table per (freqs, hd) serves every length: it
    grows (geometrically, in 512-position steps) when a longer sequence arrives, so variable-length
    training keeps O(log) tables alive instead of one per distinct length.  freqs is a persistent
    per-(dims, heads, masked, device) tensor (model.rotary_freqs).

    Streams: the processor runs dead blocks on side streams, so the stream that first needs a table is not
    the only one that reads it.  A table enters the cache only after the device has finished it and every
    earlier read of the table it replaces (a host sync, once per growth), so a read from any stream sees a
    complete table and no freed one.  Under graph
    capture (no sync possible) a missing table is built on the capturing stream, used by that one call
    and not cached (the bench warms up on the same shapes before it captures)."""
    key = (freqs.data_ptr(), int(hd), str(freqs.device))
    t = _ROT_TABLES.get(key)
    if t is not None and t.shape[0] >= L:
        return t
    cap = max(int(L), 2 * t.shape[0] if t is not None else 0)
    cap = (cap + _ROT_QUANTUM - 1) // _ROT_QUANTUM * _ROT_QUANTUM
    nt = _E(cap, int(hd) // 2, 2, device=freqs.device)
    lib.call("asrx_rotary_table", _P(freqs), _P(nt), cap, int(hd), _S())
    if torch.cuda.is_current_stream_capturing():
        return nt
    # device-wide: the side streams may still read the table this one replaces
    torch.cuda.synchronize(freqs.device)
    _ROT_TABLES[key] = nt
    return nt


def rotary(x, src, freqs, hd, scale):
    return RotaryFn.apply(x, src, freqs, hd, scale, sink_of(src), rownorm_of(src))


# =============================================================================== v_gate


class VGateFn(torch.autograd.Function):
    """v_gate.forward (model.py:346-351) -> ion (rows,) with the STE backward."""

    @staticmethod
    def forward(ctx, x, mkeyn, mval, W1, b1, W2, b2, cw, cb, tx):
        x = _c(x)
        D = x.shape[-1]
        rows = _rows(x)
        M = mkeyn.shape[0]
        Dh = W1.shape[0]
        nx = _E(rows, device=x.device)
        lib.call("asrx_rownorm", _P(x), _P(nx), rows, D, _S())
        S = G.linear_fwd(x, mkeyn)
        h = G.linear_fwd(x, W1, b1)
        ion = _E(rows, device=x.device)
        xval = _E(rows, device=x.device)
        kv = _E(rows, device=x.device)
        m2 = _E(rows, device=x.device)
        c = 1.0 / math.sqrt(D)
        lib.call("asrx_vgate_fwd", _P(S), _P(nx), _P(mval), _P(h), _P(W2), _P(b2), _P(cw), _P(cb), _P(tx), _P(ion),
                 _P(xval), _P(kv), _P(m2), rows, M, Dh, c, _S())
        ctx.dp = [_direct(ctx, i, t) for i, t in ((2, mval), (3, W1), (4, b1), (5, W2), (6, b2), (7, cw), (8, cb))]
        ctx.save_for_backward(x, mkeyn, mval, W1, W2, cw, nx, S, h, kv, m2, b1, b2, cb)
        return ion.view(*x.shape[:-1])

    @staticmethod
    def backward(ctx, gion):
        x, mkeyn, mval, W1, W2, cw, nx, S, h, kv, m2, b1, b2, cb = ctx.saved_tensors
        gion = _c(gion)
        D = x.shape[-1]
        rows = _rows(x)
        M = mkeyn.shape[0]
        Dh = W1.shape[0]
        fmval, fW1, fb1, fW2, fb2, fcw, fcb = ctx.dp
        dS = _E(rows, M, device=x.device)
        dnx = _E(rows, device=x.device)
        dh = _E(rows, Dh, device=x.device)
        dmval, dW2, db2 = _gbuf(mval, fmval), _gbuf(W2, fW2), _gbuf(b2, fb2)
        dcw, dcb = _gbuf(cw, fcw), _gbuf(cb, fcb)
        lib.call("asrx_vgate_bwd", _P(gion), _P(S), _P(nx), _P(mval), _P(h), _P(W2), _P(cw), _P(kv), _P(m2), _P(dS),
                 _P(dnx), _P(dh), _P(dmval), _P(dW2), _P(db2), _P(dcw), _P(dcb), rows, M, Dh, 1.0 / math.sqrt(D),
                 _S())
        x2 = x.view(rows, D)
        dx = G.linear_dgrad(dS, mkeyn)
        G.linear_dgrad(dh, W1, out=dx, beta=1.0)
        lib.call("asrx_rownorm_bwd", _P(dnx), _P(x2), _P(nx), _P(dx), rows, D, _S())
        dmkeyn = G.linear_wgrad(dS, x2)
        db1 = _gbuf(b1, fb1)
        dW1 = G.linear_wgrad(dh, x2, out=_gbuf(W1, fW1), accumulate=True, db=db1)
        return (dx.view(x.shape), dmkeyn, _gret(mval, dmval.view(M, 1), fmval), _gret(W1, dW1, fW1),
                _gret(b1, db1, fb1), _gret(W2, dW2.view(1, Dh), fW2), _gret(b2, db2, fb2),
                _gret(cw, dcw.view(1, 2), fcw), _gret(cb, dcb, fcb), None)


def v_gate(mod, x):
    mkeyn = torch.nn.functional.normalize(mod.mkey, p=2, dim=-1)  # parameter-sized (64 x D)
    return VGateFn.apply(x, mkeyn, mod.mval, mod.mlp[0].weight, mod.mlp[0].bias, mod.mlp[2].weight,
                         mod.mlp[2].bias, mod.concat.weight, mod.concat.bias, mod.tx)


# =============================================================================== tgate


class TGateFn(torch.autograd.Function):
    """tgate (model.py:532-535): one N=3D GEMM with sigmoid epilogue + softmax-weighted combine.  The
    three Linear(D, D) gates run as one Linear(D, 3D) over their concatenation (asrx_cat3, no ATen
    cat); the backward's concatenated weight / bias gradients land in each gate's own p.grad
    (asrx_add_segments / colsum over column blocks) instead of autograd's cat backward + adds."""

    @staticmethod
    def forward(ctx, x, W0, W1, W2, b0, b1, b2, Wcs, bcs, out_bf16=False, sink=None, osink=None, c_pre=None):
        x = _c(x)
        ctx.sink, ctx.osink = sink, osink
        ctx.set_materialize_grads(False)
        D = x.shape[-1]
        rows = _rows(x)
        def build():
            Wc, bc = _E(3 * D, D, device=x.device), _E(3 * D, device=x.device)
            lib.call("asrx_cat3", _P(W0), _P(W1), _P(W2), D * D, _P(Wc), _S())
            lib.call("asrx_cat3", _P(b0), _P(b1), _P(b2), D, _P(bc), _S())
            return Wc, bc

        Wcat, bcat = G.derived(("tgate",), build, (W0, W1, W2, b0, b1, b2))
        Gs = G.linear_fwd(x, Wcat, bcat, act="sigmoid")
        if c_pre is not None:  # cs = Linear(D, 3)(x) evaluated by the producing AbbyNormal on fp32 x
            c = c_pre
        else:
            c = _E(rows, 3, device=x.device)
            lib.call("asrx_small_linear_fwd2", _P(x), int(G.is_bf16(x)), _P(Wcs), _P(bcs), _P(c), rows, D, 3, 0, _S())
        ob = int(out_bf16 and prec.bf16_storage())
        out = _E(x.shape, device=x.device, dtype=torch.bfloat16 if ob else torch.float32)
        lib.call("asrx_tgate_fwd2", _P(Gs), _P(c), _P(out), ob, rows, D, _S())
        ctx.dWcs, ctx.dbcs = _direct(ctx, 7, Wcs), _direct(ctx, 8, bcs)
        ctx.dparts = all(_direct(ctx, k, t) for k, t in enumerate((W0, W1, W2, b0, b1, b2), 1))
        ctx.save_for_backward(x, Wcat, Wcs, Gs, c, bcs, W0, W1, W2, b0, b1, b2)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, Wcat, Wcs, Gs, c, bcs, W0, W1, W2, b0, b1, b2 = ctx.saved_tensors
        gout = grad_in(gout, ctx.osink)
        if gout is None:
            return (None,) * 13
        D = x.shape[-1]
        rows = _rows(x)
        dGz = _E(rows, 3 * D, device=x.device)
        dc = _E(rows, 3, device=x.device)
        lib.call("asrx_tgate_bwd", _P(gout), _P(Gs), _P(c), _P(dGz), _P(dc), rows, D, _S())
        if ctx.sink is not None:  # x's gradient straight into its sink (x may be bf16-stored)
            dx, acc = ctx.sink.target(x)
            G.linear_dgrad(dGz, Wcat, out=dx.view(rows, D), beta=float(acc))
        else:
            dx = G.linear_dgrad(dGz, Wcat)
        dWcs, dbcs = _gbuf(Wcs, ctx.dWcs), _gbuf(bcs, ctx.dbcs)
        lib.call("asrx_small_linear_bwd2", _P(dc), None, _P(x), int(G.is_bf16(x)), _P(Wcs), _P(dx), _P(dWcs), _P(dbcs),
                 rows, D, 3, 0, 1.0, _S())
        dWcat = _E(3 * D, D, device=x.device)
        lib.call("asrx_zero", _P(dWcat), dWcat.numel() * 4, _S())
        G.linear_wgrad(dGz, x, out=dWcat, accumulate=True)
        Ws, bs = (W0, W1, W2), (b0, b1, b2)
        if ctx.dparts:
            gw = [_gbuf(w, True) for w in Ws]
            lib.call("asrx_add_segments", _P(dWcat), D * D, _P(gw[0]), _P(gw[1]), _P(gw[2]), 3, _S())
            for k, bk in enumerate(bs):
                lib.call("asrx_colsum_ld", _P(dGz[:, k * D:]), 3 * D, _P(_gbuf(bk, True)), rows, D, _S())
            gW = [_gret(w, None, True) for w in Ws]
            gB = [_gret(bk, None, True) for bk in bs]
        else:  # not leaves (or DIRECT off): return the parts to autograd
            gW = [dWcat[k * D:(k + 1) * D] for k in range(3)]
            dbcat = colsum(dGz)
            gB = [dbcat[k * D:(k + 1) * D] for k in range(3)]
        dxr = None if ctx.sink is not None else dx.view(x.shape)
        return (dxr, *gW, *gB, _gret(Wcs, dWcs, ctx.dWcs), _gret(bcs, dbcs, ctx.dbcs), None, None, None, None)


def tgate(mod, x, out_bf16=False):
    """tgate (model.py:525-535); x fp32 or bf16-stored; out_bf16: the output only feeds a GEMM."""
    ps = [g[0].weight for g in mod.ga] + [g[0].bias for g in mod.ga] + [mod.cs[0].weight, mod.cs[0].bias]
    osink = new_sink(out_bf16) if _grad_needed(x, *ps) else None
    pre = getattr(x, "_asrx_tgate_c", None)
    c_pre = pre[0] if (pre is not None and pre[1] is mod.cs[0].weight) else None
    y = TGateFn.apply(x, *ps, out_bf16, sink_of(x), osink, c_pre)
    return out_sink(y, osink)


# =============================================================================== elementwise


class AxpyRow(torch.autograd.Function):
    """out = x + s[row] * y"""

    @staticmethod
    def forward(ctx, x, s, y):
        x, s, y = _c(x), _c(s), _c(y)
        d = x.shape[-1]
        out = _E(x.shape, device=x.device)
        lib.call("asrx_axpy_row", _P(x), _P(s), _P(y), _P(out), _rows(x), d, _S())
        ctx.save_for_backward(s, y)
        return out

    @staticmethod
    def backward(ctx, g):
        s, y = ctx.saved_tensors
        g = _c(g)
        d = y.shape[-1]
        dy = _E(y.shape, device=y.device)
        ds = _E(s.shape, device=y.device)
        lib.call("asrx_axpy_row_bwd", _P(g), _P(s), _P(y), _P(dy), _P(ds), _rows(y), d, _S())
        return g, ds, dy


def axpy_row(x, s, y):
    return AxpyRow.apply(x, s, y)


class JumpSelect(torch.autograd.Function):
    """Per-sample masked MSheath step (model.py:489-501): act ? alpha*xn + beta*orig + gam : xold."""

    @staticmethod
    def forward(ctx, xn, orig, xold, act, alpha, beta, gam):
        xn, orig, xold = _c(xn), _c(orig), _c(xold)
        act, alpha, beta, gam = _c(act), _c(alpha), _c(beta), _c(gam)
        B, L, d = xn.shape
        out = _E(xn.shape, device=xn.device)
        ctx.v4 = d % 4 == 0
        lib.call("asrx_jump_select4" if ctx.v4 else "asrx_jump_select", _P(xn), _P(orig), _P(xold), _P(act),
                 _P(alpha), _P(beta), _P(gam), _P(out), B, L, d, _S())
        ctx.save_for_backward(xn, orig, act, alpha, beta)
        return out

    @staticmethod
    def backward(ctx, g):
        xn, orig, act, alpha, beta = ctx.saved_tensors
        g = _c(g)
        B, L, d = xn.shape
        dxn, dorig, dxold = _E(xn.shape, device=g.device), _E(xn.shape, device=g.device), _E(xn.shape, device=g.device)
        if ctx.v4:  # zeroes its own accumulators
            dalpha, dbeta, dgam = _E(B, device=g.device), _E(B, device=g.device), _E(B, d, device=g.device)
        else:
            dalpha, dbeta = torch.zeros(B, device=g.device), torch.zeros(B, device=g.device)
            dgam = _E(B, d, device=g.device)
        lib.call("asrx_jump_select4_bwd" if ctx.v4 else "asrx_jump_select_bwd", _P(g), _P(xn), _P(orig), _P(act),
                 _P(alpha), _P(beta), _P(dxn), _P(dorig), _P(dxold), _P(dalpha), _P(dbeta), _P(dgam), B, L, d, _S())
        return dxn, dorig, dxold, None, dalpha, dbeta, dgam


class AxpyRow2(torch.autograd.Function):
    """out = x + s1[row] * s2[row] * y   (MSheath layer update x + g * (out * ion), model.py:461)."""

    @staticmethod
    def forward(ctx, x, s1, s2, y):
        x, s1, s2, y = _c(x), _c(s1), _c(s2), _c(y)
        d = x.shape[-1]
        out = _E(x.shape, device=x.device)
        lib.call("asrx_axpy_row2", _P(x), _P(s1), _P(s2), _P(y), _P(out), _rows(x), d, _S())
        ctx.save_for_backward(s1, s2, y)
        return out

    @staticmethod
    def backward(ctx, g):
        s1, s2, y = ctx.saved_tensors
        g = _c(g)
        d = y.shape[-1]
        dy = _E(y.shape, device=y.device)
        ds1 = _E(s1.shape, device=y.device)
        ds2 = _E(s2.shape, device=y.device)
        lib.call("asrx_axpy_row2_bwd", _P(g), _P(s1), _P(s2), _P(y), _P(dy), _P(ds1), _P(ds2), _rows(y), d, _S())
        return g, ds1, ds2, dy


_REC_BYTES = None


class MSheathCtrl(torch.autograd.Function):
    """One MSheath layer's per-sample control (model.py:461-501) as one kernel each way: potential =
    mean(ion), gumbel-hard policy -> action (forced 1 when potential < 0.1), jump weights
    alpha/beta/gam, mem_w update, next layer index.  Returns (alpha, beta, gam, mem_w_out, active,
    next_i_out); the last two carry no gradient."""

    @staticmethod
    def forward(ctx, policy, gpol_i, ion, mem_v, mem_w, mem, jump_s, next_i, layer_i, layers):
        global _REC_BYTES
        if _REC_BYTES is None:
            _REC_BYTES = int(lib.load().asrx_msheath_rec_bytes())
        policy, ion, mem_v, mem_w, mem, next_i = _c(policy), _c(ion), _c(mem_v), _c(mem_w), _c(mem), _c(next_i)
        B, L = ion.shape
        D = mem.shape[-1]
        dev = ion.device
        alpha, beta, active, next_out = (_E(B, device=dev) for _ in range(4))
        gam, mwo = _E(B, D, device=dev), _E(B, D, device=dev)
        rec = _E(B * _REC_BYTES, dtype=torch.uint8, device=dev)
        lib.call("asrx_msheath_ctrl_fwd", _P(policy), _P(gpol_i), gpol_i.stride(0), _P(ion), _P(mem_v), _P(mem_w),
                 _P(mem), _P(jump_s), _P(next_i), layer_i, layers, B, L, D, _P(alpha), _P(beta), _P(gam), _P(mwo),
                 _P(active), _P(next_out), _P(rec), _S())
        ctx.mark_non_differentiable(active, next_out)
        ctx.set_materialize_grads(False)
        ctx.djs = _direct(ctx, 6, jump_s)
        ctx.save_for_backward(mem_v, mem_w, mem, jump_s, rec)
        ctx.layer_i, ctx.layers = layer_i, layers
        return alpha, beta, gam, mwo, active, next_out

    @staticmethod
    def backward(ctx, g_alpha, g_beta, g_gam, g_mwo, _ga, _gn):
        mem_v, mem_w, mem, jump_s, rec = ctx.saved_tensors
        B, D = mem.shape
        dev = mem.device
        g_alpha = torch.zeros(B, device=dev) if g_alpha is None else _c(g_alpha)
        g_beta = torch.zeros(B, device=dev) if g_beta is None else _c(g_beta)
        g_gam = torch.zeros(B, D, device=dev) if g_gam is None else _c(g_gam)
        g_mwo = None if g_mwo is None else _c(g_mwo)
        g_policy = _E(B, 3, device=dev)
        g_mem_v = _E(mem_v.shape, device=dev)
        g_mem_w, g_mem = _E(B, D, device=dev), _E(B, D, device=dev)
        g_jump_s = _gbuf(jump_s, ctx.djs)
        lib.call("asrx_msheath_ctrl_bwd", _P(g_alpha), _P(g_beta), _P(g_gam), _P(g_mwo), _P(mem_v), _P(mem_w),
                 _P(mem), _P(jump_s), _P(rec), ctx.layer_i, ctx.layers, B, D, _P(g_policy), _P(g_mem_v), _P(g_mem_w),
                 _P(g_mem), _P(g_jump_s), _S())
        return g_policy, None, None, g_mem_v, g_mem_w, g_mem, _gret(jump_s, g_jump_s, ctx.djs), None, None, None


class SegMean(torch.autograd.Function):
    """x.mean(dim=1) for (B, L, d) -> (B, d)."""

    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        B, L, d = x.shape
        out = _E(B, d, device=x.device)
        part = _E(B * int(lib.load().asrx_mem_chunks(L)) * d, device=x.device)
        lib.call("asrx_seg_colsum_det", _P(x), _P(part), _P(out), B, L, d, 1.0 / L, _S())  # no atomics
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, g):
        B, L, d = ctx.shape
        u = _E(B, d, device=g.device)
        lib.call("asrx_lincomb", _P(_c(g)), None, None, 1.0 / L, 0.0, 0.0, _P(u), B * d, _S())
        dx = _E(B, L, d, device=g.device)
        lib.call("asrx_add_rows", None, None, _P(u), _P(dx), B, L, d, _S())
        return dx


def seg_mean(x):
    return SegMean.apply(x)


class AddRows(torch.autograd.Function):
    """out[b, l] = x[b, l] + t[l]  (t: PE table or the learned position rows)."""

    @staticmethod
    def forward(ctx, x, t, L):
        """t: the table; rows [0, L) are added (the reference's position[:T] slice)."""
        x = _c(x)
        B, Lx, d = x.shape
        out = _E(x.shape, device=x.device)
        lib.call("asrx_add_rows", _P(x), _P(t), None, _P(out), B, Lx, d, _S())
        ctx.L, ctx.d = L, d
        ctx.dt = _direct(ctx, 1, t)
        ctx.save_for_backward(t if ctx.needs_input_grad[1] else None)
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        dt = None
        if ctx.needs_input_grad[1]:
            (t,) = ctx.saved_tensors
            B = g.shape[0]
            gt = _gbuf(t, ctx.dt)
            colsum(g.view(B, -1), out=gt.view(-1)[:ctx.L * ctx.d])
            dt = _gret(t, gt, ctx.dt)
        return g, dt, None


def add_rows(x, t):
    """x (B, L, d) + t[:L] (t: a (>= L, d) table, e.g. the learned position or the sinusoid PE)."""
    L = x.shape[1]
    if t.shape[0] != L and not t.is_contiguous():
        t = t.contiguous()
    return AddRows.apply(x, t, L)


class LinComb(torch.autograd.Function):
    """out = a*x + b*y (+ c*z) with python-float coefficients."""

    @staticmethod
    def forward(ctx, x, y, z, a, b, c):
        x, y = _c(x), _c(y)
        z = _c(z) if z is not None else None
        out = _E(x.shape, device=x.device)
        lib.call("asrx_lincomb", _P(x), _P(y), _P(z), float(a), float(b), float(c), _P(out), x.numel(), _S())
        ctx.coef = (a, b, c)
        ctx.has_z = z is not None
        return out

    @staticmethod
    def backward(ctx, g):
        a, b, c = ctx.coef
        g = _c(g)

        def sc(k):
            if k == 1.0:
                return g
            out = _E(g.shape, device=g.device)
            lib.call("asrx_lincomb", _P(g), None, None, float(k), 0.0, 0.0, _P(out), g.numel(), _S())
            return out

        return sc(a), sc(b), (sc(c) if ctx.has_z else None), None, None, None


def add(x, y, z=None):
    return LinComb.apply(x, y, z, 1.0, 1.0, 1.0)


class Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        x = _c(x)
        y = _E(x.shape, device=x.device)
        lib.call("asrx_act_fwd", _P(x), _P(y), x.numel(), ACT[act], _S())
        ctx.act = act
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = _c(g)
        dx = _E(x.shape, device=x.device)
        lib.call("asrx_act_bwd", _P(g), _P(x), _P(dx), x.numel(), ACT[ctx.act], _S())
        return dx, None


def act(x, name):
    return Act.apply(x, name)


class GLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        C = x.shape[-1] // 2
        y = _E(*x.shape[:-1], C, device=x.device)
        lib.call("asrx_glu_fwd", _P(x), _P(y), _rows(x), C, _S())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dx = _E(x.shape, device=x.device)
        lib.call("asrx_glu_bwd", _P(_c(g)), _P(x), _P(dx), _rows(x), x.shape[-1] // 2, _S())
        return dx


def glu(x):
    return GLU.apply(x)


class Dropout(torch.autograd.Function):
    """nn.Dropout(p) in train mode with keyed masks on channels-last (B, T, C)."""

    @staticmethod
    def forward(ctx, x, sid_base, key, p):
        x = _c(x)
        B, T, C = x.shape
        y = _E(x.shape, device=x.device)
        lib.call("asrx_dropout", _P(x), _P(y), B, T, C, sid_base, key & 0xFFFFFFFF, float(p), _S())
        ctx.args = (sid_base, key, p)
        return y

    @staticmethod
    def backward(ctx, g):
        sid_base, key, p = ctx.args
        g = _c(g)
        B, T, C = g.shape
        dx = _E(g.shape, device=g.device)
        lib.call("asrx_dropout", _P(g), _P(dx), B, T, C, sid_base, key & 0xFFFFFFFF, float(p), _S())
        return dx, None, None, None


class ActDropout(torch.autograd.Function):
    """act, then nn.Dropout(p) in train mode, then act2 ("none" to skip) on channels-last (B, T, C),
    one kernel each way (bit-identical to Act, Dropout, Act with the same key)."""

    @staticmethod
    def forward(ctx, z, act, sid_base, key, p, act2="none"):
        z = _c(z)
        B, T, C = z.shape
        y = _E(z.shape, device=z.device)
        lib.call("asrx_act_dropout_fwd", _P(z), None, _P(y), B, T, C, sid_base, key & 0xFFFFFFFF, float(p),
                 ACT[act], ACT[act2], _S())
        ctx.args = (act, sid_base, key, p, act2)
        ctx.save_for_backward(z)
        return y

    @staticmethod
    def backward(ctx, g):
        act, sid_base, key, p, act2 = ctx.args
        (z,) = ctx.saved_tensors
        g = _c(g)
        B, T, C = z.shape
        dz = _E(z.shape, device=z.device)
        lib.call("asrx_act_dropout_bwd", _P(g), _P(z), _P(dz), B, T, C, sid_base, key & 0xFFFFFFFF, float(p),
                 ACT[act], ACT[act2], _S())
        return dz, None, None, None, None, None


class DropoutAdd(torch.autograd.Function):
    """res + nn.Dropout(p)(y) in train mode (ConvLite tail, model.py:107-118) in one pass; bit-identical
    to add(res, Dropout(y)).  Backward: d res = g, d y = the dropout of g."""

    @staticmethod
    def forward(ctx, res, y, sid_base, key, p):
        res, y = _c(res), _c(y)
        B, T, C = y.shape
        out = _E(y.shape, device=y.device)
        lib.call("asrx_act_dropout_fwd", _P(y), _P(res), _P(out), B, T, C, sid_base, key & 0xFFFFFFFF, float(p),
                 ACT["none"], ACT["none"], _S())
        ctx.args = (sid_base, key, p)
        return out

    @staticmethod
    def backward(ctx, g):
        sid_base, key, p = ctx.args
        g = _c(g)
        B, T, C = g.shape
        dy = _E(g.shape, device=g.device)
        lib.call("asrx_dropout", _P(g), _P(dy), B, T, C, sid_base, key & 0xFFFFFFFF, float(p), _S())
        return g, dy, None, None, None


def _noise_rows_ok(sid_end, C, T, k=1):
    """Keyed-noise element indices ((sid * C + c) * 8192 + t for dropout, ((sid * H + h) * 8192 + l) * 3 + k
    for the gumbel draws, oracle/keys.py) are uint32 and assume positions < 8192 (clips up to ~81.9 s
    at hop 160): refuse shapes that would alias draws instead of silently reusing them."""
    from .noise import LSTRIDE

    if T > LSTRIDE:
        raise ValueError(f"keyed noise: sequence length {T} > {LSTRIDE} positions (clips longer than ~81.9 s) "
                         "would alias dropout/gumbel draws")
    if sid_end * C * LSTRIDE * k >= 1 << 32:
        raise ValueError(f"keyed noise: {sid_end} streams x {C} channels overflow the 32-bit noise index")


def _vec4_ok(*ts):
    return all(t is None or (t.data_ptr() % 16 == 0) for t in ts) and ts[0].shape[-1] % 4 == 0


def act_dropout(z, act, sid_base, key, p, act2="none"):
    """act -> Dropout(p) -> act2 on (B, T, C): one fused float4 kernel each way, or the separate ops
    (bit-identical) when C % 4 != 0 or a tensor is not 16-byte aligned."""
    z = _c(z)
    _noise_rows_ok(sid_base + z.shape[0], z.shape[2], z.shape[1])
    if _vec4_ok(z):
        return ActDropout.apply(z, act, sid_base, key, p, act2)
    y = Dropout.apply(Act.apply(z, act) if act != "none" else z, sid_base, key, p)
    return Act.apply(y, act2) if act2 != "none" else y


def dropout_add(res, y, sid_base, key, p):
    """res + Dropout(p)(y) (ConvLite tail, model.py:107-118), fused when float4-able."""
    res, y = _c(res), _c(y)
    _noise_rows_ok(sid_base + y.shape[0], y.shape[2], y.shape[1])
    if _vec4_ok(y, res):
        return DropoutAdd.apply(res, y, sid_base, key, p)
    return add(res, Dropout.apply(y, sid_base, key, p))


class DWConv(torch.autograd.Function):
    """Depthwise Conv1d (groups=C, padding K//2) on channels-last (B, T, C); w (C, 1, K)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x = _c(x)
        B, T, C = x.shape
        K = w.shape[-1]
        y = _E(x.shape, device=x.device)
        lib.call("asrx_dwconv_fwd", _P(x), _P(w), _P(b), _P(y), B, T, C, K, _S())
        ctx.dw, ctx.db = _direct(ctx, 1, w), _direct(ctx, 2, b)
        ctx.save_for_backward(x, w, b)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, b = ctx.saved_tensors
        g = _c(g)
        B, T, C = x.shape
        K = w.shape[-1]
        dx = _E(x.shape, device=x.device)
        dw, db = _gbuf(w, ctx.dw), _gbuf(b, ctx.db)
        lib.call("asrx_dwconv_bwd", _P(g), _P(x), _P(w), _P(dx), _P(dw), _P(db), B, T, C, K, _S())
        return dx, _gret(w, dw, ctx.dw), _gret(b, db, ctx.db)


class BatchNormPS(torch.autograd.Function):
    """BatchNorm1d in train mode with per-sample statistics (batch-1 semantics) on (B, T, C)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, stats):
        x = _c(x)
        B, T, C = x.shape
        mean = _E(B, C, device=x.device)
        rstd = _E(B, C, device=x.device)
        y = _E(x.shape, device=x.device)
        lib.call("asrx_bn_fwd", _P(x), _P(w), _P(b), _P(y), _P(mean), _P(rstd), B, T, C, float(eps), 1, _S())
        if stats is not None:
            stats.append((mean, rstd))
        ctx.dw, ctx.db = _direct(ctx, 1, w), _direct(ctx, 2, b)
        ctx.save_for_backward(x, w, mean, rstd, b)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, mean, rstd, b = ctx.saved_tensors
        g = _c(g)
        B, T, C = x.shape
        sg = _E(B, C, device=x.device)
        sgx = _E(B, C, device=x.device)
        dx = _E(x.shape, device=x.device)
        dw, db = _gbuf(w, ctx.dw), _gbuf(b, ctx.db)
        lib.call("asrx_bn_bwd", _P(g), _P(x), _P(mean), _P(rstd), _P(w), _P(sg), _P(sgx), _P(dx), _P(dw), _P(db), B,
                 T, C, _S())
        return dx, _gret(w, dw, ctx.dw), _gret(b, db, ctx.db), None, None


def batch_norm_eval(x, w, b, rm, rv, eps):
    x = _c(x)
    B, T, C = x.shape
    rstd = _E(rv.shape, device=x.device)
    lib.call("asrx_rsqrt_eps", _P(_c(rv)), _P(rstd), rv.numel(), float(eps), _S())
    y = _E(x.shape, device=x.device)
    lib.call("asrx_bn_fwd", _P(x), _P(w), _P(b), _P(y), _P(_c(rm)), _P(rstd), B, T, C, float(eps), 0, _S())
    return y


class Conv3(torch.autograd.Function):
    """k3 / padding-1 Conv1d on channels-last (B, T, Cin) -> (B, T, Cout) via implicit-im2col GEMM.
    The weight is v (Cout, Cin, 3) like nn.Conv1d, weight-normed W = g v / |v| when g is given
    (weight_norm(Conv1d), model.py:140): asrx_conv3_weight writes it straight into the GEMM's k-major
    layout (bf16 in perf mode) and, for the input gradient, the flipped layout; the weight gradient
    goes back through the weight norm into g.grad / v.grad (asrx_conv3_weight_bwd)."""

    @staticmethod
    def forward(ctx, x, g, v, b, out=None):
        x = _c(x)
        B, T, Ci = x.shape
        Co = v.shape[0]
        dev = x.device
        nrm = _E(Co, device=dev) if g is not None else None
        wide = G.use_wide(3 * Ci)
        Wt = None if wide else _E(Co, 3 * Ci, device=dev)
        Wtb = _E(Co, 3 * Ci, dtype=torch.int16, device=dev) if wide else None
        lib.call("asrx_conv3_weight", _P(g), _P(_c(v)), Co, Ci, _P(Wt), _P(Wtb), None, None, _P(nrm), _S())
        y = _E(B, T, Co, device=dev) if out is None else out  # out: this stream's rows of a group buffer
        if wide:
            G.gemm_wn(x, Wtb, y, M=B * T, N=Co, K=3 * Ci, lda=Ci, ldc=Co, bias=b, conv=True, conv_F=T, conv_C=Ci)
        else:
            G.gemm(x, Wt, y, M=B * T, N=Co, K=3 * Ci, lda=Ci, ldb=3 * Ci, ldc=Co, bias=b, conv_a=True, conv_F=T,
                   conv_C=Ci)
        ctx.has_g = g is not None
        ctx.dg = _direct(ctx, 1, g) if g is not None else False
        ctx.dv, ctx.db = _direct(ctx, 2, v), _direct(ctx, 3, b)
        ctx.save_for_backward(x, g, v, b, nrm)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, g, v, b, nrm = ctx.saved_tensors
        gy = _c(gy)
        B, T, Ci = x.shape
        Co = v.shape[0]
        dev = x.device
        v = _c(v)
        dx = None
        if ctx.needs_input_grad[0]:
            wide = G.use_wide(3 * Co)
            Wf = None if wide else _E(Ci, 3 * Co, device=dev)
            Wfb = _E(Ci, 3 * Co, dtype=torch.int16, device=dev) if wide else None
            nr = _E(Co, device=dev) if g is not None else None
            lib.call("asrx_conv3_weight", _P(g), _P(v), Co, Ci, None, None, _P(Wf), _P(Wfb), _P(nr), _S())
            dx = _E(x.shape, device=dev)
            if wide:
                G.gemm_wn(gy, Wfb, dx, M=B * T, N=Ci, K=3 * Co, lda=Co, ldc=Ci, conv=True, conv_F=T, conv_C=Co)
            else:
                G.gemm(gy, Wf, dx, M=B * T, N=Ci, K=3 * Co, lda=Co, ldb=3 * Co, ldc=Ci, conv_a=True, conv_F=T,
                       conv_C=Co)
        dgo = dvo = dbo = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dWt = _E(Co, 3 * Ci, device=dev)
            lib.call("asrx_zero", _P(dWt), dWt.numel() * 4, _S())
            tiles = ((Co + 127) // 128) * ((3 * Ci + 127) // 128)
            G.gemm(gy, x, dWt, M=Co, N=3 * Ci, K=B * T, lda=Co, ldb=Ci, ldc=3 * Ci, a_kc=False, b_kc=False,
                   conv_b=True, conv_F=T, conv_C=Ci, beta=1.0, splitk=G._splitk_for(B * T, tiles))
            gv = _gbuf(v, ctx.dv) if ctx.dv else torch.zeros(v.shape, device=dev)
            gg = None
            if ctx.has_g:
                gg = _gbuf(g, ctx.dg) if ctx.dg else torch.zeros(g.shape, device=dev)
            lib.call("asrx_conv3_weight_bwd", _P(dWt), _P(g), _P(v), _P(nrm), Co, Ci, _P(gg), _P(gv), _S())
            dvo = _gret(v, gv, ctx.dv)
            dgo = _gret(g, gg, ctx.dg) if ctx.has_g else None
        if ctx.needs_input_grad[3]:
            dbo = _gret(b, colsum(gy.view(-1, Co), out=_gbuf(b, True) if ctx.db else None), ctx.db)
        return dx, dgo, dvo, dbo, None


def conv3(x, conv, out=None):
    """Conv1d(k=3, padding=1) module on channels-last x; weight_norm-parametrized modules read their
    g (original0) and v (original1) directly, so torch's parametrization kernels never run.  out: write
    into these rows of a stream-group buffer (see join_group)."""
    pz = getattr(conv, "parametrizations", None)
    if pz is not None and "weight" in pz:
        orig = pz.weight
        return Conv3.apply(x, orig.original0, orig.original1, conv.bias, out)
    return Conv3.apply(x, None, conv.weight, conv.bias, out)


class _Holder:
    __slots__ = ("buf",)

    def __init__(self, buf):
        self.buf = buf


class JoinGroup(torch.autograd.Function):
    """The stream-group buffer whose row blocks the parts were written into (the encoder stems of the
    equal-length audio streams, AudioEncoder.encode): the group enters the shared encoder pass without a
    concatenation copy (was torch.cat: 590 MB of HBM traffic per step at the tiny config); the
    backward hands each part its rows of the group gradient (views, no copy)."""

    @staticmethod
    def forward(ctx, holder, *parts):
        ctx.set_materialize_grads(False)
        ctx.n, ctx.B = len(parts), parts[0].shape[0]
        return holder.buf

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None,) * (ctx.n + 1)
        B = ctx.B
        return (None,) + tuple(g[i * B:(i + 1) * B] for i in range(ctx.n))


def join_group(buf, parts):
    """buf (n B, ...) whose row blocks are exactly `parts` (written in place by their producers)."""
    for i, t in enumerate(parts):
        B = t.shape[0]
        assert t.data_ptr() == buf[i * B].data_ptr() and t.shape[1:] == buf.shape[1:], "parts must be buf's rows"
    if not (torch.is_grad_enabled() and any(t.requires_grad for t in parts)):
        return buf
    return JoinGroup.apply(_Holder(buf), *parts)


class Stem1(torch.autograd.Function):
    """Conv1d(1, D, 3, padding=1) (model.py:133) on (B, T) single-channel streams -> (B, T, D)."""

    @staticmethod
    def forward(ctx, x, W, b, out=None):
        x = _c(x)
        B, T = x.shape
        D = W.shape[0]
        y = _E(B, T, D, device=x.device) if out is None else out  # out: rows of a stream-group buffer
        lib.call("asrx_stem1_fwd", _P(x), _P(W), _P(b), _P(y), B, T, D, _S())
        ctx.dW, ctx.db = _direct(ctx, 1, W), _direct(ctx, 2, b)
        ctx.save_for_backward(x, W, b)
        return y

    @staticmethod
    def backward(ctx, g):
        x, W, b = ctx.saved_tensors
        B, T = x.shape
        D = W.shape[0]
        dW, db = _gbuf(W, ctx.dW), _gbuf(b, ctx.db)
        lib.call("asrx_stem1_bwd", _P(_c(g)), _P(x), _P(dW), _P(db), B, T, D, _S())
        return None, _gret(W, dW, ctx.dW), _gret(b, db, ctx.db), None


class Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, E):
        ids = _c(ids)
        d = E.shape[1]
        y = _E(*ids.shape, d, device=E.device)
        lib.call("asrx_embed_fwd", _P(ids), _P(E), _P(y), ids.numel(), d, _S())
        ctx.dE = _direct(ctx, 1, E)
        ctx.save_for_backward(ids, E if ctx.dE else None)
        ctx.Eshape = E.shape
        return y

    @staticmethod
    def backward(ctx, g):
        ids, E = ctx.saved_tensors
        dE = _gbuf(E, True) if ctx.dE else torch.zeros(ctx.Eshape, device=g.device)
        lib.call("asrx_embed_bwd", _P(ids), _P(_c(g)), _P(dE), ids.numel(), ctx.Eshape[1], _S())
        return None, _gret(E, dE, ctx.dE)


class CrossEntropy(torch.autograd.Function):
    """F.cross_entropy(logits, labels, ignore_index=0), mean over non-ignored rows (model.py:670):
    one read of the logits (online log-sum-exp), the mean and the non-ignored count on the device;
    the backward scale g / count is read on the device (no host sync, graph-capturable)."""

    @staticmethod
    def forward(ctx, logits, labels):
        z = _c(logits)
        V = z.shape[-1]
        rows = _rows(z)
        lab = _c(labels.reshape(-1))
        loss_r = _E(rows, device=z.device)
        lse = _E(rows, device=z.device)
        loss = _E((), device=z.device)
        count = _E(1, device=z.device)
        lib.call("asrx_ce_fwd1", _P(z), _P(lab), _P(loss_r), _P(lse), _P(loss), _P(count), rows, V, _S())
        ctx.save_for_backward(z, lab, lse, count)
        return loss

    @staticmethod
    def backward(ctx, g):
        z, lab, lse, count = ctx.saved_tensors
        g = _c(g.reshape(1).to(torch.float32)) if g.dtype != torch.float32 or not g.is_contiguous() else g
        dz = _E(z.shape, device=z.device)
        lib.call("asrx_ce_bwd2", _P(z), _P(lab), _P(lse), _P(g), _P(count), _P(dz), _rows(z), z.shape[-1], _S())
        return dz, None


class LogitsCE(torch.autograd.Function):
    """Tied logits + F.cross_entropy(logits, labels, ignore_index=0) fused (perf mode with bf16 storage;
    model.py:629 logits = x @ token.weight^T, model.py:670 the loss).  One GEMM writes the logits -- fp32,
    the boundary's dtype (model.py:629 .float()), or bf16 when opted in -- and, per row and column tile,
    the (max, sum exp) of the stored logits; a per-row merge gives the log-sum-exp and the loss, reading
    only the label's logit.  The backward writes dz = (g/count)(softmax - onehot) bf16 from the stored
    logits and feeds it to the
    input-gradient GEMM and the embedding's weight-gradient GEMM.  The logits stay an output with a
    gradient path (a gradient arriving for them is added to dz)."""

    @staticmethod
    def forward(ctx, h, W, labels, sink, bf16_logits=False):
        h = _c(h)
        ctx.set_materialize_grads(False)
        ctx.sink = sink
        rows, D = _rows(h), h.shape[-1]
        V = W.shape[0]
        nj = G._nj(rows, V)
        nparts = (V + 128 * nj - 1) // (128 * nj)
        zb = _E(*h.shape[:-1], V, dtype=torch.bfloat16 if bf16_logits else torch.float32, device=h.device)
        part = _E(rows, nparts, 2, device=h.device)
        Wb = G.weight_bf16(W)
        lib.require_gpu(h, Wb, zb)
        e0 = probe.begin("gemm")
        lib.call("asrx_gemm_wn_ce" if bf16_logits else "asrx_gemm_wn_ce_f32", _P(h), D, _P(Wb), Wb.stride(0), _P(zb),
                 V, _P(part), rows, V, D, nj, _S())
        probe.end("gemm", e0, 2.0 * rows * V * D,
                  ("wn", rows, V, D, nj, 0, "none", False, False, 1, int(bf16_logits), -1))
        lab = _c(labels.reshape(-1))
        loss_r = _E(rows, device=h.device)
        lse = _E(rows, device=h.device)
        loss = _E((), device=h.device)
        count = _E(1, device=h.device)
        lib.call("asrx_ce_part_fwd" if bf16_logits else "asrx_ce_part_fwd_f32", _P(part), nparts, _P(zb), _P(lab),
                 _P(loss_r), _P(lse), _P(loss), _P(count), rows, V, _S())
        ctx.dW = _direct(ctx, 1, W)
        ctx.save_for_backward(h, W, zb, lab, lse, count)
        return zb, loss

    @staticmethod
    def backward(ctx, g_logits, g_loss):
        h, W, zb, lab, lse, count = ctx.saved_tensors
        rows, V = _rows(zb), zb.shape[-1]
        if g_loss is None:
            g_loss = torch.zeros(1, device=zb.device)
        g_loss = _c(g_loss.reshape(1).float())
        dz = _E(zb.shape, dtype=torch.bfloat16, device=zb.device)
        lib.call("asrx_ce_bwd_bf16" if zb.dtype == torch.bfloat16 else "asrx_ce_bwd_f32in", _P(zb), _P(lab), _P(lse),
                 _P(g_loss), _P(count), _P(dz), rows, V, _S())
        if g_logits is not None:  # a gradient for the logits themselves (not the training path)
            dz = dz.float() + g_logits.float()
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.sink is not None:
                buf, acc = ctx.sink.target(h)
                G.linear_dgrad(dz, W, out=buf, beta=float(acc))
            else:
                dx = G.linear_dgrad(dz, W)
        dW = None
        if ctx.needs_input_grad[1]:
            gW = _gbuf(W, ctx.dW)
            G.linear_wgrad(dz, h, out=gW, accumulate=True)
            dW = _gret(W, gW, ctx.dW)
        return dx, dW, None, None, None


def logits_ce_ok(h, W) -> bool:
    """The fused tied-logits + cross entropy applies: perf mode with the final norm stored bf16."""
    return (h.dtype == torch.bfloat16 and W.dim() == 2 and W.shape[0] % 8 == 0 and h.shape[-1] % 8 == 0
            and prec.get() == prec.PREC_BF16)


def logits_ce(h, W, labels, bf16_logits=False):
    """(logits, loss) = (h W^T, F.cross_entropy(., labels, ignore_index=0)) through LogitsCE; the logits are
    fp32 (model.py:629 returns .float() logits) unless bf16_logits (opt-in: half the logits bytes)."""
    return LogitsCE.apply(h, W, labels, sink_of(h), bool(bf16_logits))


class BlendFn(torch.autograd.Function):
    """sigmoid(blend) d + (1 - sigmoid(blend)) g (processor output, model.py:628)."""

    @staticmethod
    def forward(ctx, d, g, blend):
        d, g = _c(d), _c(g)
        out = _E(d.shape, device=d.device)
        lib.call("asrx_blend_fwd", _P(d), _P(g), _P(blend), _P(out), d.numel(), _S())
        ctx.db = _direct(ctx, 2, blend)
        ctx.save_for_backward(d, g, blend)
        return out

    @staticmethod
    def backward(ctx, go):
        d, g, blend = ctx.saved_tensors
        go = _c(go)
        dd = _E(d.shape, device=d.device) if ctx.needs_input_grad[0] else None
        dg = _E(g.shape, device=g.device) if ctx.needs_input_grad[1] else None
        dbl = None
        if ctx.needs_input_grad[2]:
            dbl = _gbuf(blend, ctx.db)
        lib.call("asrx_blend_bwd", _P(go), _P(d), _P(g), _P(blend), _P(dd), _P(dg), _P(dbl), d.numel(), _S())
        return dd, dg, (_gret(blend, dbl, ctx.db) if dbl is not None else None)


def blend(d, g, b):
    return BlendFn.apply(d, g, b)


def policy_noise(B, layers, sid_base, key, device):
    out = _E(B, layers, 3, device=device)
    lib.call("asrx_policy_noise", _P(out), B, layers, sid_base, key & 0xFFFFFFFF, _S())
    return out
