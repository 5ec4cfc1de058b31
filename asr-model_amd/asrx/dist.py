"""Data-parallel gradient synchronisation: bucketed all-reduce overlapped with backward
(SURVEY.md §8(e)).  One process per GPU, torch.distributed with backend "nccl" (= RCCL on ROCm)
over xGMI; "gloo" works the same way on CPU for the tests.

Design (MI355X-first, not a translation of DDP's call pattern):
  * the bucket plan covers exactly the parameters that receive gradients in this model (found on
    the first step: dead blocks, the unused attn.c / rot.lin / router / span_scale / pitch_tokens
    never do), in reverse registration order = roughly the order backward produces them;
  * gradients live in the flat bucket buffers (p.grad is a view), so no copy is needed;
  * readiness is counted in gradient events: autograd's post-accumulate-grad hook, and each
    contribution the asrx kernels accumulate straight into p.grad (asrx.ops.GRAD_LISTENERS).  How
    many events a parameter receives depends on how the step was batched (asrx Model runs equal-
    length audio streams as one pass, so a pitch track whose length differs from the spectrogram's
    means one more pass per shared weight).  The counts are therefore learned PER STEP SIGNATURE
    (`model.grad_signature`, set by Model.forward: the stream lengths): a step with a new signature
    counts its events and reduces every bucket in finish(); a step with a known signature launches a
    bucket's all-reduce as soon as the bucket has seen all of its events -- a comm stream waits on
    the compute stream and the all-reduce then runs under the rest of backward;
  * an event that arrives after its bucket's all-reduce was launched means the launch read a
    partial gradient: that raises (it cannot happen while event counts are a function of the
    signature, and the check keeps it from ever passing silently);
  * finish() joins the comm stream; buckets a step left incomplete are reduced there with their
    missing slots zero (variable unused parameters);
  * bucket size defaults to 64 MB: one 8-GPU ring step over 7 xGMI links moves bucket/8 per link
    per step, large enough that per-call latency is amortised at the 96 MB (tiny) .. 1 GB (medium)
    payloads, small enough that the first bucket launches early in backward.
"""
from __future__ import annotations

import weakref

import torch
import torch.distributed as dist

from . import ops


class _Bucket:
    __slots__ = ("params", "buf", "pending", "expected", "work", "launched", "offsets")

    def __init__(self, params, device):
        self.params = params
        n = sum(p.numel() for p in params)
        self.buf = torch.zeros(n, device=device, dtype=torch.float32)
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p.numel()
        self.expected = self.pending = len(params)
        self.work = None
        self.launched = False


class GradSync:
    def __init__(self, model: torch.nn.Module, bucket_mb: float = 64.0, group=None, signature=None,
                 reduce_single: bool = False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # reduce_single: run the bucket all-reduces even in a 1-rank group (exercises the RCCL launch,
        # comm-stream overlap and join on a one-GPU box; the sum over one rank is the identity)
        self.active = self.world > 1 or (reduce_single and dist.is_initialized())
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.bucket_bytes = int(bucket_mb * 1024 * 1024)
        self.buckets: list[_Bucket] | None = None
        self.where: dict[int, tuple[_Bucket, int]] = {}
        dev = self.params[0].device
        self.cuda = dev.type == "cuda"
        self.comm = torch.cuda.Stream(device=dev) if self.cuda else None
        self.hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        # step signature -> learned gradient events per parameter (id) / per bucket
        self._signature = signature if signature is not None else (lambda: getattr(model, "grad_signature", None))
        self.plans: dict = {}
        self.bucket_plans: dict = {}
        self._reset_step()
        self._listener = weakref.WeakMethod(self._ready)
        ops.GRAD_LISTENERS.append(self._listener)

    def _reset_step(self):
        self._seen: dict[int, int] = {}  # events of the current step per parameter
        self._sig = None
        self._started = False
        self._overlap = False  # this step launches buckets from the hooks (known signature)

    # ------------------------------------------------------------------ plan
    def _build(self):
        live = [p for p in self.params if p.grad is not None]
        buckets, cur, size = [], [], 0
        for p in reversed(live):
            cur.append(p)
            size += p.numel() * 4
            if size >= self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        dev = live[0].device
        self.buckets = [_Bucket(ps, dev) for ps in buckets]
        for b in self.buckets:
            for p, off in zip(b.params, b.offsets):
                self.where[id(p)] = (b, off)
                b.buf[off:off + p.numel()].copy_(p.grad.reshape(-1))
                p.grad = b.buf[off:off + p.numel()].view_as(p)

    def _learn(self, sig):
        """Record this step's event counts as the plan of its signature."""
        self.plans[sig] = dict(self._seen)
        self.bucket_plans[sig] = [sum(max(1, self._seen.get(id(p), 0)) for p in b.params) for b in self.buckets]

    def zero_grad(self):
        """Zero the bucket buffers (the grads are views of them) before the next backward."""
        self._reset_step()
        if self.buckets is None:
            for p in self.params:
                p.grad = None
            return
        for b in self.buckets:
            b.buf.zero_()
            b.work = None
            b.launched = False
            for p, off in zip(b.params, b.offsets):
                if p.grad is None or p.grad.data_ptr() != b.buf[off:].data_ptr():
                    p.grad = b.buf[off:off + p.numel()].view_as(p)

    # ------------------------------------------------------------------ overlap
    def _start_step(self):
        self._started = True
        self._sig = self._signature()
        plan = self.bucket_plans.get(self._sig)
        self._overlap = self.buckets is not None and plan is not None and self.active
        if self._overlap:
            for b, n in zip(self.buckets, plan):
                b.expected = b.pending = n

    def _ready(self, p):
        if not self._started:
            self._start_step()
        self._seen[id(p)] = self._seen.get(id(p), 0) + 1
        if not self._overlap:
            return
        entry = self.where.get(id(p))
        if entry is None:
            return
        b = entry[0]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)
        elif b.pending < 0:
            raise RuntimeError(
                "GradSync: a gradient event arrived after its bucket's all-reduce was launched (step "
                f"signature {self._sig!r} delivered more events than the learned plan); the all-reduce read a "
                "partial gradient")

    def _launch(self, b: _Bucket):
        if b.launched:
            return
        b.launched = True
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(ev)
                b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        """Join every bucket's all-reduce and average.  Call after backward, before the optimizer."""
        if not self._started:
            self._start_step()
        if self.buckets is None:
            self._build()  # first step: nothing overlapped yet
        if self._sig not in self.bucket_plans:
            self._learn(self._sig)
        elif self._overlap:
            plan = self.plans[self._sig]
            extra = [i for i, n in self._seen.items() if n > plan.get(i, 0)]
            if extra:  # would have raised in _ready for an overlapped bucket; a bucket not yet launched is fine
                self.plans[self._sig] = {i: max(n, self._seen.get(i, 0)) for i, n in plan.items()} | \
                    {i: n for i, n in self._seen.items() if i not in plan}
                self._learn(self._sig)
        if self.active:
            for b in self.buckets:
                if not b.launched:
                    self._launch(b)
            for b in self.buckets:
                b.work.wait()
            if self.cuda:
                torch.cuda.current_stream().wait_stream(self.comm)
            inv = 1.0 / self.world
            for b in self.buckets:
                b.buf.mul_(inv)
        self._reset_step()

    def remove(self):
        for h in self.hooks:
            h.remove()
        if self._listener in ops.GRAD_LISTENERS:
            ops.GRAD_LISTENERS.remove(self._listener)


def broadcast_parameters(model: torch.nn.Module, src: int = 0):
    """Replicas start from rank 0's parameters and buffers."""
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)
