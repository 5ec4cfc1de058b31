"""Live per-kernel timing for bench.py: HIP events recorded around selected launches on the stream
they run on (torch.cuda.Event on torch's current stream, which is the stream every asrx launch
uses).  Off unless a bench enables it."""
from __future__ import annotations

import torch

_active: dict | None = None
_precise = 0


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
