"""GEMM entry points over ``asrx_gemm`` (csrc/gemm.hip) for Linear / Conv1d forward and backward.

Layout vocabulary: activations are row-major (rows, features); weights are nn.Linear's (out, in).
"""
from __future__ import annotations

import torch

from . import lib, prec, probe

ACT = {"none": 0, "gelu": 1, "silu": 2, "sigmoid": 3, "relu": 4}


BF16 = torch.bfloat16


def is_bf16(t) -> bool:
    return t is not None and t.dtype == BF16


def gemm(A, B, C, *, M, N, K, lda, ldb, ldc, a_kc=True, b_kc=True, batch=1, sA=0, sB=0, sC=0,
         bias=None, Z=None, alpha=1.0, beta=0.0, act="none", conv_a=False, conv_b=False,
         conv_F=0, conv_C=0, splitk=1, precision=None):
    """The generic fp32-storage GEMM (csrc/gemm.hip): every operand fp32 in HBM."""
    lib.require_gpu(A, B, C)
    if is_bf16(A) or is_bf16(B) or is_bf16(C):
        raise RuntimeError("asrx_gemm takes fp32 operands; bf16-stored activations go through the wide GEMM")
    p = prec.get() if precision is None else precision
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm", p, lib.ptr(A), lda, sA, int(a_kc), int(conv_a), lib.ptr(B), ldb, sB,
             int(b_kc), int(conv_b), lib.ptr(C), ldc, sC, lib.ptr(bias), lib.ptr(Z), M, N, K, batch,
             float(alpha), float(beta), ACT[act], conv_F, conv_C, int(splitk), lib.stream())
    probe.end("gemm", e0, 2.0 * M * N * K * batch,
              ("gemm", p, M, N, K, batch, int(a_kc), int(b_kc), int(conv_a), splitk, act))
    return C


def _rows(x):
    return x.reshape(-1, x.shape[-1])


# ------------------------------------------------------------------ wide-N activation x weight GEMM
# bf16 copies of the weights used in this step (asrx_weight_to_bf16), keyed by storage, layout and
# version; cleared at the start of every Model.forward so that updated weights are re-converted and
# the conversions of a step stay inside that step (and inside its captured graph).
#
# Bulk plan: the parameter weights (and views of them) a step converted are recorded; from the next
# step on, clear_weight_cache converts all of them in ONE launch (asrx_weights_to_bf16, ~200
# launches fewer per tiny step) into a persistent arena on the current stream, at the start of the
# forward -- before any side stream forks -- so the entries serve every stream.  Weights derived per
# step (tgate's concatenation, v_gate's normalised keys) keep the lazy per-call conversion.
_WCACHE: dict = {}
_BULK: dict = {}       # (ptr, shape, stride, trans) -> (source, bf16 arena view), valid for the current step
_SEEN: dict = {}       # plan being recorded for the current owner: key -> (source tensor,)
_PLANS: dict = {}      # id(owner model) -> (keys, sources, arena views, table, max_elems)
_OWNER = None          # id of the model whose step is running (set by clear_weight_cache)
_PLAN_OFF = False


def _bulk_key(W, trans):
    return (W.data_ptr(), tuple(W.shape), tuple(W.stride()), bool(trans))


def _is_param_weight(W):
    base = W._base if W._base is not None else W
    return isinstance(base, torch.nn.Parameter) and W.is_cuda and W.stride(1) == 1


def _build_plan():
    if not _SEEN:
        return None
    keys = list(_SEEN)
    srcs = [_SEEN[k][0] for k in keys]
    _SEEN.clear()
    sizes = [t.numel() for t in srcs]
    dev = srcs[0].device
    arena = torch.empty(sum(sizes), dtype=torch.int16, device=dev)
    import numpy as np
    nb = int(lib.load().asrx_wconv_entry_bytes())
    rec = np.zeros(len(keys), dtype=np.dtype([("src", "<u8"), ("dst", "<u8"), ("ld", "<i8"), ("rows", "<i4"),
                                              ("cols", "<i4"), ("trans", "<i4"), ("pad", "<i4")]))
    assert rec.dtype.itemsize == nb, (rec.dtype.itemsize, nb)
    views, off = [], 0
    for i, (k, W) in enumerate(zip(keys, srcs)):
        rows, cols = W.shape
        trans = k[3]
        v = arena[off:off + W.numel()].view((cols, rows) if trans else (rows, cols))
        rec[i] = (W.data_ptr(), v.data_ptr(), W.stride(0), rows, cols, int(trans), 0)
        views.append(v)
        off += W.numel()
    table = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
    return (keys, srcs, views, table, max(sizes))


# weights derived from parameters per step (tgate's concatenation, v_gate's combined projection), built
# once per step and stream by their first user: parameters do not change inside a step, so the 7 calls
# of one block's tgate (and the dead blocks' calls on the side streams) share one build per stream
_DERIVED: dict = {}


def derived(key, build, refs=()):
    """The per-step cached value of `key` on the current stream (build() makes it on first use).  refs: the
    tensors the value is derived from; their addresses, shapes and versions join the key and the entry holds
    them, so their memory cannot be recycled for another tensor that would then hit a stale entry of a
    different shape (a standalone module used without end_step() -- the MSheath op test after a smaller
    one -- read such an entry out of bounds)."""
    k = (key, tuple((t.data_ptr(), tuple(t.shape), t._version) for t in refs),
         torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0)
    v = _DERIVED.get(k)
    if v is None:
        v = build()
        _DERIVED[k] = (v, tuple(refs))
        return v
    return v[0]


def end_step():
    """End of a step (the backward, or a forward without one): drop the per-step copies.  The bulk
    views are keyed by parameter address; once a step is over the parameters may be freed (their model
    dropped) and another tensor allocated at the same address must not find them."""
    _WCACHE.clear()
    _BULK.clear()
    _DERIVED.clear()


def clear_weight_cache(owner=None):
    """Start of a step of `owner` (a Model): drop the per-step copies, then convert the weights this
    owner's previous steps used in one launch (its plan is recorded during its first wide step)."""
    global _OWNER
    _WCACHE.clear()
    _BULK.clear()
    _DERIVED.clear()
    capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    if _OWNER is not None and _SEEN and _OWNER not in _PLANS and not capturing:
        _PLANS[_OWNER] = _build_plan()  # the previous step of that owner recorded its weights
        # (never built inside a graph capture: the table upload is a synchronous copy)
    _SEEN.clear()
    _OWNER = id(owner) if owner is not None else None
    if _PLAN_OFF or _OWNER is None:
        return
    plan = _PLANS.get(_OWNER)
    if plan is None:
        if _OWNER not in _PLANS:
            import weakref
            weakref.finalize(owner, _PLANS.pop, _OWNER, None)
        return
    keys, srcs, views, table, mx = plan
    if not all(t.data_ptr() == k[0] for t, k in zip(srcs, keys)):  # parameters were reallocated
        del _PLANS[_OWNER]
        return
    lib.call("asrx_weights_to_bf16", lib.ptr(table), len(keys), mx, lib.stream())
    # the entries hold their source weights: until the next clear their memory cannot be recycled for another
    # tensor that would hit a stale entry (a model dropped after its forward, then ops on new weights: the
    # fused-residual test after the model tests read the dropped model's bf16 copy)
    _BULK.update((k, (s, v)) for k, s, v in zip(keys, srcs, views))


def plan_token():
    """Identity of the running step's bulk bf16 arena (None before its owner's plan exists): a recorded launch
    sequence that reads the arena's views (a dead-block graph) is valid only while this token is unchanged."""
    plan = _PLANS.get(_OWNER) if _OWNER is not None else None
    return None if not plan or not plan[2] else (_OWNER, plan[2][0].data_ptr())


def plan_refs():
    """The tensors of the running step's bulk plan (arena views, entry table): held by a graph that reads them."""
    plan = _PLANS.get(_OWNER) if _OWNER is not None else None
    return () if not plan else tuple(plan[2]) + (plan[3],)


def forget_stream(stream_id):
    """Drop the per-step cache entries made on one stream (after a graph capture on it: their values live in the
    graph's pool and hold the right contents only after a replay)."""
    for d in (_WCACHE, _DERIVED):
        for k in [k for k in d if k[-1] == stream_id]:
            del d[k]


def weight_bf16(W, trans=False, cache=True):
    """bf16 N x K copy of a weight: W is (N, K) (trans=False) or (K, N) (trans=True).  Cached per
    stream: a copy converted on one stream is never read by another before it is complete."""
    if cache and _BULK:
        hit = _BULK.get(_bulk_key(W, trans))
        if hit is not None:
            return hit[1]
    key = (W.data_ptr(), tuple(W.shape), tuple(W.stride()), bool(trans), W._version,
           torch.cuda.current_stream(W.device).cuda_stream if W.is_cuda else 0) if cache else None
    if key is not None and key in _WCACHE:
        return _WCACHE[key][1]
    src = W
    rows, cols = W.shape
    if W.stride(1) != 1:
        W = W.contiguous()
    out = torch.empty((cols, rows) if trans else (rows, cols), dtype=torch.int16, device=W.device)
    lib.call("asrx_weight_to_bf16", lib.ptr(W), lib.ptr(out), rows, cols, W.stride(0), int(trans), lib.stream())
    if key is not None:
        # the entry holds the source tensor too, so its address cannot be recycled for another
        # tensor (which would alias the key) while the entry lives
        _WCACHE[key] = (src, out)
        if _OWNER is not None and _PLANS.get(_OWNER) is None and not _PLAN_OFF and _is_param_weight(src):
            _SEEN.setdefault(_bulk_key(src, trans), (src,))
    return out


_nj_override = None


# Minimum tile counts (in 128 x 128 nj units) for the 384- and 256-column tile widths.  Large activations (the audio
# side, >= 16384 rows): the widest width that still gives >= 200 tiles.  Below that (the text side's 2048-8192-row
# launches) a wider tile wins with fewer tiles: nj = 3 from 180, nj = 2 from 144 (profiles/r06_small_m_nj_sweep_*.txt:
# 45 text-side shapes, 1099 -> ~1025 us summed, e.g. 2048 x 3072 x 1024 37.0 -> 26.5 us, 8192 x 768 x 384 18.8 ->
# 14.7 us).  Every tile width runs the same k order per output element, so the products are bit-identical.
NJ_MIN_TILES = {"large": (200, 200), "small": (180, 144)}


def _nj(M, N, a_bf16=True):
    """Tile width 128*nj of the persistent wide GEMM (NJ_MIN_TILES); narrow tiles run two workgroups per CU.  An fp32
    activation whose N leaves the last 384-wide tile partly empty takes the 256-wide tile (N = M + Dh of the MSheath
    product: 448 at small, 576 at medium -- 48016 x 448 x 768 93 -> 69 us, 24000 x 576 x 1024 74 -> 52 us; a bf16
    activation is within 3 % either way, profiles/r06_nj_pad.txt)."""
    if _nj_override:
        return _nj_override
    tm = (M + 127) // 128
    t3, t2 = NJ_MIN_TILES["large" if M >= 16384 else "small"]
    for nj, th in ((3, t3), (2, t2)):
        if nj == 3 and not a_bf16 and N % 384:
            continue
        if 128 * nj <= ((N + 127) // 128) * 128 and tm * ((N + 128 * nj - 1) // (128 * nj)) >= th:
            return nj
    return 1


# Plain bf16-activation products go to the vendor library (hipBLASLt, asrx_gemm_lt) where it measured faster than the
# wide GEMM: K >= 768 at >= 16384 rows, 25-40 % (profiles/r06_blaslt_vs_wide.txt); every fused epilogue, fp32
# activations, row-tile lists and K = 384 stay on the hand-written kernels.  False: the wide GEMM everywhere.
LIBRARY_GEMM = __import__("os").environ.get("ASRX_LIBRARY_GEMM", "1") != "0"
LIB_MIN_K, LIB_MIN_M = 768, 16384


def _lib_ok(A, Wb, C, M, N, K, lda, ldc, Z, act, conv, mtiles, beta):
    return (LIBRARY_GEMM and is_bf16(A) and not conv and mtiles is None and act == "none" and Z is None
            and K >= LIB_MIN_K and M >= LIB_MIN_M and (beta == 0.0 or not is_bf16(C))
            and A.data_ptr() % 16 == 0 and Wb.data_ptr() % 16 == 0 and C.data_ptr() % 16 == 0)


def gemm_wn(A, Wb, C, *, M, N, K, lda, ldc, bias=None, Z=None, alpha=1.0, beta=0.0, act="none",
            conv=False, conv_F=0, conv_C=0, mtiles=None):
    """C = act(alpha A Wb^T + beta C + bias); Wb bf16 (N, K) from weight_bf16.  A and C are stored fp32
    or bf16 (their dtype; a bf16 C takes beta = 0); mtiles: only these 128-row tiles (row_tiles).  Plain
    bf16-A products at the library's shapes run on hipBLASLt (LIBRARY_GEMM)."""
    lib.require_gpu(A, Wb, C)
    ab, cb = int(is_bf16(A)), int(is_bf16(C))
    if _lib_ok(A, Wb, C, M, N, K, lda, ldc, Z, act, conv, mtiles, beta):
        e0 = probe.begin("gemm")
        lib.call("asrx_gemm_lt", lib.ptr(A), lda, lib.ptr(Wb), Wb.stride(0), lib.ptr(C), cb, ldc, lib.ptr(bias), M, N,
                 K, float(alpha), float(beta), lib.stream())
        probe.end("gemm", e0, 2.0 * M * N * K, ("lt", M, N, K, cb, beta != 0))
        return C
    nj = _nj(M, N, ab)
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm_wn_ex", lib.ptr(A), ab, lda, int(conv), conv_F, conv_C, lib.ptr(Wb), Wb.stride(0),
             lib.ptr(C), cb, ldc, lib.ptr(bias), lib.ptr(Z), M, N, K, float(alpha), float(beta), ACT[act], nj,
             lib.ptr(mtiles[0]) if mtiles is not None else None, lib.ptr(mtiles[1]) if mtiles is not None else None,
             lib.stream())
    # row-list launches: the tag carries a probe snapshot of the device-built tile count (-1: all rows)
    rl = probe.keep(mtiles[1]) if (mtiles is not None and probe.active()) else (-1 if mtiles is None else -2)
    probe.end("gemm", e0, 2.0 * M * N * K,
              ("wn", M, N, K, nj, int(conv), act, Z is not None, beta != 0, ab, cb, rl))
    return C


RECOMPUTE_ACT = True  # Linear + act in perf mode: the backward recomputes the pre-activation (gemm_wn_gact)
# Measured per forward + backward (tools/microbench.py gact, profiles/r04_gact_micro.txt): SiLU at
# 192064 x 1536 1602 -> 1531 us and 8192 x 1536 147 -> 139 us, but 96000 x 1536 715 -> 759 us; GELU at
# 192064 x 1152 1200 -> 1264 us (erf and exp inside the one-workgroup-per-CU GEMM's epilogue hold the
# MFMA pipeline).  The recompute saves the pre-activation's HBM round trip (2 x 4 bytes per element) but is
# time-neutral overall, so it is used for SiLU / sigmoid and not for GELU.
RECOMPUTE_ACTS = ("silu", "sigmoid")


def can_recompute_act(x, W, act):
    """True when Linear(x, W) + act may skip storing its pre-activation: perf mode, silu / sigmoid, and
    the shape the activation-gradient GEMM covers (the forward's tile width nj = 3, aligned rows)."""
    if not RECOMPUTE_ACT or act not in RECOMPUTE_ACTS or not x.is_cuda:
        return False
    N, K = W.shape[0], W.shape[-1] if W.dim() == 2 else W.numel() // W.shape[0]
    M = x.numel() // max(K, 1)
    return (use_wide(K) and use_wide(N) and N % 8 == 0 and M > 0 and _nj(M, N) == 3
            and (not is_bf16(x) or K % 8 == 0))


def linear_gact(x, W, b, gy, gz, act, db=None):
    """gz (bf16, gy's shape) = gy * act'(x W^T + b), the pre-activation recomputed by the GEMM; db (fp32, N)
    += column sums of gz when given.  x as the forward saw it (fp32 or bf16-stored)."""
    x2 = _rows(x)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = W.shape[0]
    Wb = weight_bf16(W.view(N, -1))
    g2 = gy.reshape(M, N)
    if g2.dtype != torch.float32 or not g2.is_contiguous():
        g2 = g2.float().contiguous()
    nj = _nj(M, N)
    lib.require_gpu(x2, Wb, g2, gz)
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm_wn_gact", lib.ptr(x2), int(is_bf16(x2)), K, lib.ptr(Wb), Wb.stride(0), lib.ptr(b),
             lib.ptr(g2), N, lib.ptr(gz), N, lib.ptr(db), M, N, K, ACT[act], nj, lib.stream())
    probe.end("gemm", e0, 2.0 * M * N * K, ("gact", M, N, K, nj, act, int(is_bf16(x2))))
    return gz


def router_fwd(x2, W1, b1, W2, keep_hpre):
    """AbbyNormal router in one GEMM pass: (hpre or None, logits (M, 3) without b2)."""
    M, K = x2.shape
    N = W1.shape[0]
    Wb = weight_bf16(W1)
    hpre = torch.empty(M, N, device=x2.device) if keep_hpre else None
    logits = torch.empty(M, 3, device=x2.device)
    lib.require_gpu(x2, Wb, logits)
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm_wn_router", lib.ptr(x2), K, lib.ptr(Wb), Wb.stride(0), lib.ptr(b1), lib.ptr(W2),
             lib.ptr(hpre), N, lib.ptr(logits), M, N, K, lib.stream())
    probe.end("gemm", e0, 2.0 * M * N * K, ("router", M, N, K, keep_hpre))
    return hpre, logits


def use_wide(K) -> bool:
    return prec.get() == prec.PREC_BF16 and K % 8 == 0


def gemm_wn_rows(A, Wb, C, *, M, N, K, lda, ldc, mtiles, bias=None, alpha=1.0, beta=0.0):
    """gemm_wn on the 128-row tiles listed on the device (mtiles = (list, count) from row_tiles)."""
    return gemm_wn(A, Wb, C, M=M, N=N, K=K, lda=lda, ldc=ldc, bias=bias, alpha=alpha, beta=beta, mtiles=mtiles)


def row_tiles(next_i, layer, L, M, device=None):
    """(list, count) of the 128-row tiles of an M-row activation holding rows of samples at MSheath
    layer `layer` (next_i[b] == layer, L rows per sample), built on the device.  next_i: a tensor, or a device
    address with `device` given."""
    n = int(lib.load().asrx_row_tiles_max(M))
    dev = device if device is not None else next_i.device
    tl = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    lib.call("asrx_row_tiles", lib.ptr(next_i), layer, L, M, lib.ptr(tl), lib.ptr(cnt), lib.stream())
    return tl, cnt


def linear_fwd(x, W, b=None, act="none", out=None, preact=None, wbf=None, mtiles=None, out_bf16=False):
    """y = act(x @ W^T + b) for x (..., K) (fp32 or bf16-stored), W (N, K); wbf: W's bf16 copy when the
    caller made it; mtiles: only these 128-row tiles (perf mode; the fp32 parity GEMM computes every
    row); out_bf16: store y bf16 (perf mode, when y only feeds GEMM operands)."""
    x2 = _rows(x)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = W.shape[0]
    wide = use_wide(K)
    if is_bf16(x2) and not wide:
        x2 = x2.float()  # the fp32 GEMM (parity mode / K % 8 != 0) reads fp32
    odt = BF16 if (out_bf16 and wide and N % 4 == 0) else torch.float32
    y = out if out is not None else torch.empty(*x.shape[:-1], N, device=x.device, dtype=odt)
    if wide and mtiles is not None and act == "none" and preact is None:
        gemm_wn_rows(x2, weight_bf16(W) if wbf is None else wbf, y, M=M, N=N, K=K, lda=K, ldc=N, bias=b,
                     mtiles=mtiles)
    elif use_wide(K):
        gemm_wn(x2, weight_bf16(W) if wbf is None else wbf, y, M=M, N=N, K=K, lda=K, ldc=N, bias=b, act=act,
                Z=preact)
    else:
        gemm(x2, W, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, a_kc=True, b_kc=True, bias=b, act=act,
             Z=preact)
    return y


def linear_rot_fwd(x, W, b, m, tab, L, hd, scale, preact=None):
    """rotary(x @ W^T + b) in one wide GEMM (perf mode, asrx_gemm_wn_rot): x (B, L, K) fp32 or bf16-stored, W
    (N, K), m (B L,) the rotary magnitudes (||src|| per row), tab the (cos, sin) table of rotary_table;
    preact (B, L, N) fp32 receives the unrotated product when given.  -> (B, L, N) fp32."""
    x2 = _rows(x)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = W.shape[0]
    Wb = weight_bf16(W)
    y = torch.empty(*x.shape[:-1], N, device=x.device)
    nj = _nj(M, N)
    ab = int(is_bf16(x2))
    lib.require_gpu(x2, Wb, y, m, tab)
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm_wn_rot", lib.ptr(x2), ab, K, lib.ptr(Wb), Wb.stride(0), lib.ptr(y), lib.ptr(preact), N,
             lib.ptr(b), lib.ptr(m), lib.ptr(tab), L, hd, float(scale), M, N, K, nj, lib.stream())
    probe.end("gemm", e0, 2.0 * M * N * K, ("wn", M, N, K, nj, 0, "rot", preact is not None, False, ab, 0, -1))
    return y


def linear_dgrad(dy, W, out=None, beta=0.0, mtiles=None):
    """dx = dy @ W (fp32 dx)."""
    """dx = dy @ W for dy (..., N), W (N, K); mtiles as in linear_fwd."""
    d2 = _rows(dy)
    if not d2.is_contiguous():
        d2 = d2.contiguous()
    M, N = d2.shape
    K = W.shape[1]
    dx = out if out is not None else torch.empty(*dy.shape[:-1], K, device=dy.device, dtype=torch.float32)
    if use_wide(N) and mtiles is not None:
        gemm_wn_rows(d2, weight_bf16(W, trans=True), dx, M=M, N=K, K=N, lda=N, ldc=K, beta=beta, mtiles=mtiles)
    elif use_wide(N):
        gemm_wn(d2, weight_bf16(W, trans=True), dx, M=M, N=K, K=N, lda=N, ldc=K, beta=beta)
    else:
        gemm(d2, W, dx, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, a_kc=True, b_kc=False, beta=beta)
    return dx


def _splitk_for(m_rows: int, tiles: int) -> int:
    # about 512 workgroups (two per CU, all resident: the measured optimum at 192k rows); each K
    # slice keeps >= 256 rows (text-side 8192-row shapes: 32 slices ran 34 us vs 38 us at 16)
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, m_rows // 256)))


# bias gradients summed inside the weight-gradient kernel (False: a separate column-sum pass; the
# fusion test compares the two on a whole model)
FUSED_BIAS_GRAD = True
# tests: a list makes every fused bias sum also take the column sums of the SAME dY in a separate pass and
# append (fused contribution, column sums) -- the fusion checked inside one backward
BIAS_CHECK = None


def _wgrad(A, lda, x2, out, M, K, rows, db=None):
    """out (M, K) += A^T x2 over `rows` rows (A: (rows, >= M) with row stride lda, x2: (rows, K), fp32 or
    bf16-stored); db (M,): += the column sums of A (the bias gradient) -- in the same kernel pass on the
    register-staged paths (asrx_wgrad_bias), a column-sum pass otherwise."""
    tiles = ((M + 127) // 128) * ((K + 127) // 128)
    sk = _splitk_for(rows, tiles)

    def staged(a_bf16, b_bf16, name, *tag):
        lib.require_gpu(A, x2, out)
        e0 = probe.begin("gemm")
        if db is not None and not FUSED_BIAS_GRAD:
            staged_db, db_ = db, None
        else:
            staged_db, db_ = None, db
        if db_ is not None:
            before = db_.clone() if BIAS_CHECK is not None else None
            lib.call("asrx_wgrad_bias", lib.ptr(A), a_bf16, lda, lib.ptr(x2), b_bf16, K, lib.ptr(out), out.stride(0),
                     lib.ptr(db), M, K, rows, sk, lib.stream())
            if before is not None:
                Af = A.float() if a_bf16 else A
                ref = torch.zeros(M, device=A.device)
                lib.call("asrx_colsum_ld", lib.ptr(Af), Af.stride(0) if a_bf16 else lda, lib.ptr(ref), rows, M,
                         lib.stream())
                absum = Af.as_strided((rows, M), (Af.stride(0) if a_bf16 else lda, 1)).abs().sum(0)
                # allowed difference: fp32 summation order (1e-5 of the column's sum of |dY|) plus the rounding
                # of the += into what the bias gradient already held (2 ulp)
                tol = 1e-5 * absum + 2.0 ** -22 * (before.abs() + ref.abs())
                BIAS_CHECK.append((db_ - before, ref, tol, dict(M=M, K=K, rows=rows, sk=sk, a_bf16=a_bf16,
                                                                  b_bf16=b_bf16, lda=lda, ldo=out.stride(0))))
        elif name == "asrx_wgrad_bf16":
            lib.call(name, lib.ptr(A), lda, lib.ptr(x2), K, lib.ptr(out), out.stride(0), M, K, rows, sk, lib.stream())
        else:
            lib.call(name, lib.ptr(A), lda, lib.ptr(x2), b_bf16, K, lib.ptr(out), out.stride(0), M, K, rows, sk,
                     lib.stream())
        probe.end("gemm", e0, 2.0 * M * K * rows, ("wgrad", M, K, rows, sk) + tag)
        if staged_db is not None:  # unfused reference: column sums of dY (fp32 copy when bf16-stored)
            Af = A.float() if a_bf16 else A
            lib.call("asrx_colsum_ld", lib.ptr(Af), Af.stride(0) if a_bf16 else lda, lib.ptr(staged_db), rows, M,
                     lib.stream())
        return out

    if is_bf16(A):
        # a bf16-stored dY (the tied logits' gradient from the fused cross entropy, an activation's bf16
        # gradient from asrx_act_bwd_bias); X fp32 or bf16
        xb = is_bf16(x2)
        if M % 8 or K % (8 if xb else 4) or lda % 8 or x2.stride(0) != K or A.data_ptr() % 16 or x2.data_ptr() % 16:
            A = A.float()  # contiguous copy (of a column-slice view too): its own row stride
            lda = A.stride(0)
        else:
            return staged(1, int(xb), "asrx_wgrad_bf16_ab", 2 + int(xb))
    if is_bf16(x2):
        # a bf16-stored activation: the register-staged bf16 kernel at every shape (its X bytes halve)
        if M % 4 or K % 8 or lda % 4 or x2.stride(0) != K or A.data_ptr() % 16:
            x2 = x2.float()
        else:
            return staged(0, 1, "asrx_wgrad_bf16_ex", 1)
    ok4 = M % 4 == 0 and K % 4 == 0 and lda % 4 == 0 and A.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0
    # register-staged bf16 kernel with transpose reads (csrc/gemm_wg.hip): faster where the output
    # has few tiles (D x D weights, 1.2-2.6x on the 8192-row text side); the wide 1152/1536 outputs at
    # 192k rows stay on the split-K LDS-DMA kernel (5-12 % faster there, tools/wgrad_bench.py); at 24-48k rows
    # (small / medium B=8) every output up to 72 tiles is 5-25 % faster on the staged kernel, 768 x 3072 is not
    # (profiles/r06_wgrad_bench.txt)
    if prec.get() == prec.PREC_BF16 and ok4 and x2.stride(0) == K and (tiles <= 9 or rows <= 16384
                                                                        or (rows <= 50000 and tiles <= 72)):
        return staged(0, 0, "asrx_wgrad_bf16")
    gemm(A, x2, out, M=M, N=K, K=rows, lda=lda, ldb=K, ldc=K, a_kc=False, b_kc=False, beta=1.0, splitk=sk)
    if db is not None:
        lib.call("asrx_colsum_ld", lib.ptr(A), lda, lib.ptr(db), rows, M, lib.stream())
    return out


def wgrad_cols(dy, c0, n, x, out):
    """out (n, K) += dy[:, c0:c0+n]^T @ x for row-major dy (rows, ld) and x (rows, K): the weight
    gradient of one column block of a GEMM output, read in place (no copy of the block)."""
    rows, ld = dy.shape
    return _wgrad(dy[:, c0:], ld, x, out, n, x.shape[1], rows)


def linear_wgrad(dy, x, out=None, accumulate=False, db=None):
    """dW = dy^T @ x (N, K) summed over all rows; accumulates into `out` when accumulate=True.  db (N,):
    the bias gradient, += column sums of dy (fused into the weight-gradient pass where it can be)."""
    d2 = _rows(dy)
    x2 = _rows(x)
    if not d2.is_contiguous():
        d2 = d2.contiguous()
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, N = d2.shape
    K = x2.shape[1]
    if out is None:
        out = torch.zeros(N, K, device=dy.device, dtype=torch.float32)
    elif not accumulate:
        out.zero_()
    return _wgrad(d2, N, x2, out, N, K, M, db=db)
