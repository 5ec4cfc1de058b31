"""MaxFactor optimizer and FAMScheduler2 (optimizerc.py:6-147, 770-795) with the same constructor
signatures, parameter-group semantics and state names, so the reference's setup (model.py:772-791:
group 1 = every parameter, 'bias': 1.0; group 2 = names containing jump / pnet / micro_filter,
'bias': 2.0) drops in unchanged.

The step itself is one native call (``asrx_maxfactor_step``, csrc/maxfactor.hip) over every
parameter that has a gradient: eight kernel launches for the whole model, no per-parameter host
sync.  The reference reads four scalars back per parameter (.item()); here the only host work is
updating the cached parameter table (step counts, beta_t / rho_t, lr) and one asynchronous H2D copy.
Deliberate difference: ``state["RMS"]`` (written by the reference, never read) is not kept.
``clip=True`` (off in the reference configuration) is not implemented and raises.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import lib


# one parameter record, byte-compatible with MFParam in csrc/maxfactor.hip (144 bytes)
_REC = np.dtype([("p", "u8"), ("g", "u8"), ("rv", "u8"), ("cv", "u8"), ("v", "u8"), ("n", "i8"), ("mats", "i4"),
                 ("rows", "i4"), ("cols", "i4"), ("mode", "i4"), ("beta", "f4"), ("rho", "f4"), ("lr", "f4"),
                 ("decay", "f4"), ("gamma", "f4"), ("d", "f4"), ("eps1", "f4"), ("eps2", "f4"), ("row0", "i8"),
                 ("cc0", "i8"), ("col0", "i8"), ("mat0", "i8"), ("item0", "i8"), ("gsz", "i4"),
                 ("pad_", "i4")])


_CHUNK = 256  # rows per column-sum work item (MF_CHUNK)


def _group(length: int) -> int:
    """Lanes per row in the row kernels: the power of two >= the row length, at most a wave (64)."""
    g = 1
    while g < min(length, 64):
        g *= 2
    return g


def _geometry(p: torch.Tensor):
    """(mats, rows, cols) of the reference's factored view: rows reduce over the last dim, columns
    over dim -2, leading dims are independent matrices (row_var (..., R, 1), col_var (..., 1, C))."""
    if p.dim() <= 1:  # vectors and 0-d scalars (e.g. blend / threshold parameters)
        return 1, 1, p.numel()
    rows, cols = p.shape[-2], p.shape[-1]
    return p.numel() // (rows * cols), rows, cols


class MaxFactor(torch.optim.Optimizer):
    __version__ = "1.0"

    def __init__(self, params, lr=0.025, b_decay=-0.8, eps=(1e-8, 1e-8), d=1.0, decay=0.01, gamma=0.99, max=False,
                 bias=1, min_lr=1e-9, clip=False, cap=0.0):
        defaults = dict(lr=lr, b_decay=b_decay, eps=eps, d=d, decay=decay, gamma=gamma, max=max, bias=bias,
                        min_lr=min_lr, clip=clip, cap=cap)
        super().__init__(params=params, defaults=defaults)
        self._ws = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        live = []  # (group, p, grad)
        for group in self.param_groups:
            if group["clip"]:
                raise NotImplementedError("MaxFactor(clip=True) is not implemented (off in the reference setup)")
            for p in group["params"]:
                if p.grad is None:
                    continue
                lib.require_gpu(p, p.grad)
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise ValueError("MaxFactor expects contiguous float32 parameters")
                grad = p.grad if p.grad.dtype == torch.float32 and p.grad.is_contiguous() else p.grad.float().contiguous()
                if group["max"]:
                    grad = -grad
                live.append((group, p, grad))
        if not live:
            return loss
        key = tuple((id(g), p.data_ptr(), gr.data_ptr()) for g, p, gr in live)
        if getattr(self, "_key", None) != key:
            self._build(live)
            self._key = key
        c = self._cache
        # per-step scalars, vectorised over the table (steps advance together for every live param)
        torch._foreach_add_(c["step_tensors"], 1.0)
        c["steps"] += 1.0
        tab = c["tab"]
        tab["lr"] = np.array([g["lr"] for g, _, _ in live], dtype=np.float32)
        tab["beta"] = c["steps"] ** c["b_decay"]
        tab["rho"] = np.maximum(c["min_lr"], np.minimum(tab["lr"], 1.0 / np.sqrt(c["steps"])))
        # asynchronous H2D of the table from two alternating pinned buffers: a buffer is rewritten
        # only after the copy that read it two steps ago has completed
        k = c["flip"] = c["flip"] ^ 1
        c["done"][k].synchronize()
        c["pinned"][k].numpy()[:] = tab.view(np.uint8)
        c["dev_tab"][k].copy_(c["pinned"][k], non_blocking=True)
        c["done"][k].record()
        lib.call("asrx_maxfactor_step", c["dev_tab"][k].data_ptr(), len(live), c["nrows"], c["ncols"], c["ncc"],
                 c["nmats"], c["nitems"], c["ws"].data_ptr(), lib.stream())
        self._keep = [gr for _, _, gr in live]  # asynchronous call: keep converted gradients alive
        return loss

    def _build(self, live):
        lib_ = lib.load()
        if _REC.itemsize != lib_.asrx_maxfactor_param_bytes():
            raise RuntimeError("MaxFactor record layout does not match libasrx")
        tab = np.zeros(len(live), dtype=_REC)
        nrows = ncols = ncc = nmats = nitems = 0
        steps, b_decay, min_lr, step_tensors = [], [], [], []
        for i, (group, p, grad) in enumerate(live):
            eps1, eps2 = group["eps"]
            if eps1 is None:
                eps1 = torch.finfo(torch.float32).eps
            state = self.state[p]
            if len(state) == 0:  # optimizerc.py:39-46
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                if p.dim() > 1:
                    rs, cs = list(p.shape), list(p.shape)
                    rs[-1], cs[-2] = 1, 1
                    state["row_var"], state["col_var"] = p.new_zeros(rs), p.new_zeros(cs)
                state["v"] = torch.zeros_like(p)
            mats, rows, cols = _geometry(p)
            mode = 0 if p.dim() <= 1 else (1 if (p.dim() < 3 or group["bias"] == 1) else 2)
            gsz = _group(p.numel() if mode == 0 else cols)
            tab[i] = (p.data_ptr(), grad.data_ptr(), lib.ptr(state.get("row_var")) or 0,
                      lib.ptr(state.get("col_var")) or 0, state["v"].data_ptr(), p.numel(), mats, rows, cols, mode,
                      0.0, 0.0, group["lr"], group["decay"], group["gamma"], group["d"], eps1, eps2, nrows, ncc, ncols,
                      nmats, nitems, gsz, 0)
            nitems += -(-(1 if mode == 0 else mats * rows) // (64 // gsz))
            if mode == 0:
                nrows += 1
            else:
                nrows += mats * rows
                ncols += mats * cols
                ncc += mats * cols * ((rows + _CHUNK - 1) // _CHUNK)
                nmats += mats
            steps.append(float(state["step"]))
            b_decay.append(group["b_decay"])
            min_lr.append(group["min_lr"])
            step_tensors.append(state["step"])
        device = live[0][1].device
        self._cache = dict(tab=tab, nrows=nrows, ncols=ncols, ncc=ncc, nmats=nmats, nitems=nitems, device=device,
                           steps=np.array(steps, dtype=np.float64), b_decay=np.array(b_decay, dtype=np.float64),
                           min_lr=np.array(min_lr, dtype=np.float64), step_tensors=step_tensors,
                           ws=torch.empty(4 * len(live) + 4 * nrows + ncols + nmats, device=device,
                                          dtype=torch.float32),
                           pinned=[torch.empty(tab.nbytes, dtype=torch.uint8).pin_memory() for _ in range(2)],
                           dev_tab=[torch.empty(tab.nbytes, dtype=torch.uint8, device=device) for _ in range(2)],
                           done=[torch.cuda.Event(), torch.cuda.Event()], flip=0)


class FAMScheduler2(torch.optim.lr_scheduler.LRScheduler):
    """optimizerc.py:770-795: linear warmup from warmup_start, hold until decay_start, then cosine to
    eta_min (+1e-8)."""

    def __init__(self, optimizer, warmup_steps=1000, total_steps=100000, decay_start=10, warmup_start=1e-6,
                 eta_min=1e-6, last_epoch=-1):
        self.warmup_steps = warmup_steps
        self.total_steps = total_steps
        self.decay_start_step = decay_start if decay_start is not None else warmup_steps
        self.warmup_start_lr = warmup_start
        self.eta_min = eta_min
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        if self.last_epoch < self.warmup_steps:
            a = self.last_epoch / self.warmup_steps
            return [self.warmup_start_lr + (b - self.warmup_start_lr) * a for b in self.base_lrs]
        if self.last_epoch < self.decay_start_step:
            return list(self.base_lrs)
        frac = (self.last_epoch - self.decay_start_step) / (self.total_steps - self.decay_start_step)
        return [self.eta_min + (b - self.eta_min) * (1 + math.cos(math.pi * frac)) / 2 + 1e-8 for b in self.base_lrs]


def reference_param_groups(model: torch.nn.Module):
    """model.py:772-781: the two MaxFactor groups of the reference training script."""
    main, jump = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (jump if ("jump" in name or "pnet" in name or "micro_filter" in name) else main).append(p)
    return [{"params": main, "bias": 1.0}, {"params": jump, "bias": 2.0}]
