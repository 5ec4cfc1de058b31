"""Live per-kernel timing for bench.py: HIP events recorded around selected launches on the stream
they run on (torch.cuda.Event on torch's current stream, which is the stream every asrx launch
uses).  Off unless a bench enables it."""
from __future__ import annotations

import torch

_active: dict | None = None
_precise = 0
_aux: list = []  # device values a tag refers to by index (read back after the probed step)


def enable(kinds=("gemm", "logmel", "attn"), precise_cycles=0):
    """precise_cycles > 0: a spin kernel of that many cycles (torch.cuda._sleep) runs before every timed
    launch, so the host has enqueued the start event, the launch and the end event before the GPU reaches
    them -- in an eager step small kernels otherwise include the host's launch latency (tools/
    gemm_table.py)."""
    global _active, _precise
    _active = {k: [] for k in kinds}
    _precise = int(precise_cycles)


def disable():
    global _active
    out, _active = _active, None
    return out


def active():
    return _active is not None


def keep(t):
    """Snapshot a small device tensor (stream-ordered clone) for a tag; -> its index (aux(i) after a sync).
    The row-list GEMMs take their row-tile count from the device, so their bytes are known only after the
    step: the probe keeps a copy of the count as it was at the launch."""
    _aux.append(t.clone())
    return len(_aux) - 1


def aux(i):
    return _aux[i]


def clear_aux():
    _aux.clear()


def begin(kind):
    if _active is None or kind not in _active:
        return None
    if _precise:
        torch.cuda._sleep(_precise)
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def end(kind, e0, work, tag=None):
    if e0 is None:
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    _active[kind].append((work, e0, e1, tag))


def summarize(records):
    """-> (launches, total work, total seconds); call after a device synchronize."""
    n, work, sec = 0, 0.0, 0.0
    for w, e0, e1, _ in records:
        n += 1
        work += w
        sec += e0.elapsed_time(e1) * 1e-3
    return n, work, sec


def by_tag(records):
    """-> {tag: (launches, total work, total seconds)}; call after a device synchronize."""
    out: dict = {}
    for w, e0, e1, tag in records:
        n, wk, sec = out.get(tag, (0, 0.0, 0.0))
        out[tag] = (n + 1, wk + w, sec + e0.elapsed_time(e1) * 1e-3)
    return out


def _rows_of(M, rl):
    """Rows a wide-GEMM launch computes: all M, or the device-built row-tile count kept at the launch."""
    if rl == -1 or rl is False:
        return M
    if rl is True or rl < 0:
        return None  # a row-list launch made while the probe was off: unknown
    return min(M, int(aux(rl).item()) * 128)


def gemm_wr_bytes(tag):
    """Algorithmic HBM bytes of one gemm_wr_kernel launch (every instantiation: plain / residual / tied
    logits, router, activation-gradient) from its probe tag; None for the other GEMM kernels.  Counted once
    each: A (4 B fp32 or 2 B bf16-stored per element; a k3 conv's implicit im2col reads each activation row
    once, so K/3 of it), the bf16 weight (2 N K), C written (4 / 2 B), C or the residual read again
    (beta / RES), the saved fp32 pre-activation; router: logits 3 x 4 B per row (+ h_pre when kept);
    activation-gradient: G read (4 B) and gz written (2 B) per output element."""
    kind = tag[0] if tag else None
    if kind == "wn":
        _, M, N, K, _nj, conv, _act, has_z, has_beta, ab, cb, rl = tag
        rows = _rows_of(M, rl)
        if rows is None:
            return None
        ea, ec = (2 if ab else 4), (2 if cb else 4)
        ka = K // 3 if conv else K
        return ea * rows * ka + 2 * N * K + ec * rows * N * (1 + int(has_beta)) + 4 * rows * N * int(has_z)
    if kind == "router":
        _, M, N, K, keep_hpre = tag
        return 4 * M * K + 2 * N * K + 12 * M + 4 * M * N * int(keep_hpre)
    if kind == "gact":
        _, M, N, K, _nj, _act, ab = tag
        return (2 if ab else 4) * M * K + 2 * N * K + 6 * M * N
    return None


def gemm_flops(tag, work):
    """The probe's flop count of a GEMM launch, corrected for row-list launches (only their tiles' rows)."""
    if tag and tag[0] == "wn":
        M, rl = tag[1], tag[11]
        rows = _rows_of(M, rl)
        if rows is not None and M > 0:
            return work * rows / M
    return work
