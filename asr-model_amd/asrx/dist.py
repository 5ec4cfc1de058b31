"""Data-parallel gradient synchronisation: bucketed all-reduce overlapped with backward
(the seam is the reference's backward -> optimizer step, essentials.py:772-821).
One process per GPU, torch.distributed with backend "nccl" (= RCCL on ROCm) over xGMI; "gloo" works
the same way on CPU for the tests.

Design (MI355X-first, not a translation of DDP's call pattern):
  * gradients live in flat bucket buffers (p.grad is a view), so no copy is needed;
  * the bucket plan covers every parameter that CAN receive a gradient -- `model.grad_reachable()`
    when the model declares it (asrx Model: everything but the dead blocks and the unused attn.c /
    rot.lin / router / span_scale / pitch_tokens), every requires_grad parameter otherwise -- plus
    whatever received one on the first step; a covered parameter that gets no gradient in a step is
    reduced as zeros, so one that first receives a gradient on a later step is still
    reduced and zeroed like the rest.  The layout is made identical on every rank: the live masks are
    max-reduced and rank 0's backward completion
    order (the order in which each parameter took its last gradient of that step) is broadcast, so
    bucket 0 holds what backward finishes first (the processor) and the last bucket the encoder;
  * the first bucket is small (bucket_mb / 4) so the first all-reduce starts early in backward;
  * COLLECTIVE ORDER IS RANK-INDEPENDENT BY CONSTRUCTION: bucket i is launched only after buckets
    0..i-1 (the next-bucket rule): a bucket that completes early waits for its predecessors, and
    finish() launches whatever is left in index order.  Every rank therefore issues the same
    sequence of all-reduces of the same sizes, whether it launched them from backward hooks (a
    known step signature) or from finish() (a new one), so ranks that see different signatures in
    the same step -- DataCollator pads each rank's batch to its own maximum -- cannot pair buckets
    of different sizes or hang;
  * readiness is counted in gradient events: autograd's post-accumulate-grad hook, and each
    contribution the asrx kernels accumulate straight into p.grad (asrx.ops.GRAD_LISTENERS).  How
    many events a parameter receives depends on how the step was batched (equal-length audio
    streams share one pass), so the counts are learned PER STEP SIGNATURE (`model.grad_signature`:
    the train flag and the stream GROUPING, not raw lengths, so variable-length data keeps one
    signature per grouping and overlap engages);
  * an event that arrives after its bucket's all-reduce was launched means the launch read a
    partial gradient: that raises (it cannot happen while event counts are a function of the
    signature, and the check keeps it from ever passing silently);
  * finish() joins the comm stream; buckets a step left incomplete are reduced there with their
    missing slots zero (variable unused parameters);
  * BatchNorm running statistics (model.py:103 BatchNorm1d in ConvLite) are training state outside the
    gradient: each rank's forward updates its own, so finish() also averages every floating-point
    running_mean / running_var over the ranks (one small flat all-reduce behind the last bucket) and the
    replicas' eval-mode outputs stay identical (DDP instead rebroadcasts rank 0's buffers each step);
  * opt-in bf16 wire format (comm_dtype=torch.bfloat16): a bucket is rounded to bf16 into its own comm
    buffer on the comm stream, all-reduced as bf16 (half the bytes over xGMI: medium's ~1 GB of gradient per step
    becomes ~0.5 GB) and widened back to fp32 before the average.  The gradients stay fp32 everywhere else;
    the rounding adds ~2^-9 relative error per element and rank (tests/test_dist.py bounds it against fp32).
"""
from __future__ import annotations

import weakref

import torch
import torch.distributed as dist

from . import ops


class _Bucket:
    __slots__ = ("params", "buf", "pending", "expected", "work", "launched", "complete", "offsets", "cbuf")

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
        self.complete = False
        self.cbuf = None  # bf16 wire copy (GradSync comm_dtype=torch.bfloat16)


class GradSync:
    def __init__(self, model: torch.nn.Module, bucket_mb: float = 64.0, group=None, signature=None,
                 reduce_single: bool = False, first_bucket_mb: float | None = None, cover=None,
                 comm_dtype=torch.float32):
        """cover: the parameters that can receive a gradient (default: model.grad_reachable() if the
        model declares it, else every requires_grad parameter); each gets a bucket slot from step 1.
        comm_dtype: the all-reduce's wire format, torch.float32 (default) or torch.bfloat16 (opt-in)."""
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"GradSync comm_dtype must be torch.float32 or torch.bfloat16, got {comm_dtype}")
        self.comm_dtype = comm_dtype
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # reduce_single: run the bucket all-reduces even in a 1-rank group (exercises the RCCL launch,
        # comm-stream overlap and join on a one-GPU box; the sum over one rank is the identity)
        self.active = self.world > 1 or (reduce_single and dist.is_initialized())
        self.params = [p for p in model.parameters() if p.requires_grad]
        if cover is None:
            cover = model.grad_reachable() if hasattr(model, "grad_reachable") else self.params
        self._cover = {id(p) for p in cover if p.requires_grad}
        self.bucket_bytes = int(bucket_mb * 1024 * 1024)
        fb = bucket_mb / 4 if first_bucket_mb is None else first_bucket_mb
        self.first_bucket_bytes = int(fb * 1024 * 1024)
        self.buckets: list[_Bucket] | None = None
        self.where: dict[int, tuple[_Bucket, int]] = {}
        dev = self.params[0].device
        self.cuda = dev.type == "cuda"
        self.device = dev
        self.comm = torch.cuda.Stream(device=dev) if self.cuda else None
        self.hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        # step signature -> learned gradient events per parameter (id) / per bucket
        self._signature = signature if signature is not None else (lambda: getattr(model, "grad_signature", None))
        self.plans: dict = {}
        self.bucket_plans: dict = {}
        self._last_event: dict[int, int] = {}  # first step: event clock of each parameter's last event
        self._clock = 0
        self._reset_step()
        self._listener = weakref.WeakMethod(self._ready)
        ops.GRAD_LISTENERS.append(self._listener)
        # per step: how many buckets the backward hooks launched and how many were left to finish() (a bucket whose
        # learned plan has no event holds back every later bucket under the next-bucket rule) -- the
        # last step's counts, and per known signature the largest number its overlapped steps left to finish()
        self.last_overlap = None
        self.left_to_finish: dict = {}
        self._stat_bufs = [b for n, b in model.named_buffers()
                           if b.is_floating_point() and n.rsplit(".", 1)[-1] in ("running_mean", "running_var")]
        self._stat_flat = None

    def _reset_step(self):
        self._seen: dict[int, int] = {}  # events of the current step per parameter
        self._sig = None
        self._started = False
        self._overlap = False  # this step launches buckets from the hooks (known signature)
        self._next = 0  # index of the next bucket to launch (buckets launch strictly in index order)

    # ------------------------------------------------------------------ plan
    def _agree_layout(self, live_idx, order_key):
        """Rank-identical live set and parameter order: the union of the ranks' live masks, ordered by
        rank 0's backward completion (ties and parameters rank 0 did not see: reverse registration)."""
        n = len(self.params)
        comm_dev = self.device if (self.cuda and dist.get_backend(self.group) == "nccl") else torch.device("cpu")
        mask = torch.zeros(n, dtype=torch.int32, device=comm_dev)
        mask[live_idx] = 1
        key = torch.tensor([order_key.get(i, 1 << 40) for i in range(n)], dtype=torch.int64, device=comm_dev)
        if self.world > 1 or self.active:
            dist.all_reduce(mask, op=dist.ReduceOp.MAX, group=self.group)
            src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
            dist.broadcast(key, src, group=self.group)
        mask, key = mask.cpu().tolist(), key.cpu().tolist()
        live = [i for i in range(n) if mask[i]]
        return sorted(live, key=lambda i: (key[i], -i))

    def _build(self):
        live_idx = [i for i, p in enumerate(self.params) if p.grad is not None or id(p) in self._cover]
        order = {i: self._last_event.get(id(self.params[i]), 1 << 40) for i in live_idx}
        if dist.is_initialized() and (self.world > 1 or self.active):
            idx = self._agree_layout(live_idx, order)
        else:
            idx = sorted(live_idx, key=lambda i: (order[i], -i))
        buckets, cur, size = [], [], 0
        for i in idx:
            p = self.params[i]
            cur.append(p)
            size += p.numel() * 4
            if size >= (self.first_bucket_bytes if not buckets else self.bucket_bytes):
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        self.buckets = [_Bucket(ps, self.device) for ps in buckets]
        for b in self.buckets:
            for p, off in zip(b.params, b.offsets):
                self.where[id(p)] = (b, off)
                if p.grad is not None:
                    b.buf[off:off + p.numel()].copy_(p.grad.reshape(-1))
                p.grad = b.buf[off:off + p.numel()].view_as(p)
        self._last_event.clear()

    def _learn(self, sig, counts):
        """Record `counts` (events per parameter id) as the plan of signature `sig`."""
        self.plans[sig] = dict(counts)
        # a covered parameter with no event in this signature adds nothing to its bucket's count (a bucket
        # of such parameters is complete -- all zeros -- as soon as the step starts)
        self.bucket_plans[sig] = [sum(counts.get(id(p), 0) for p in b.params) for b in self.buckets]

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
            b.complete = False
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
                # a bucket the plan gives no event is NOT launched from the hooks: under the same signature
                # a parameter of it may still take its first gradient later in this step (an event after
                # the launch would mean a partial reduce); finish() launches it, and by the next-bucket
                # rule the buckets behind it, once backward is done
                b.complete = False

    def _ready(self, p):
        if not self._started:
            self._start_step()
        self._seen[id(p)] = self._seen.get(id(p), 0) + 1
        if self.buckets is None:  # first step: remember the completion order for the bucket layout
            self._clock += 1
            self._last_event[id(p)] = self._clock
        if not self._overlap:
            return
        entry = self.where.get(id(p))
        if entry is None:
            return
        b = entry[0]
        b.pending -= 1
        if b.pending == 0:
            b.complete = True
            self._launch_ready()
        elif b.pending < 0 and not b.launched:
            # more events than the learned plan for a bucket still waiting on an earlier one (the
            # next-bucket rule): nothing read it yet -- finish() launches it in index order and merges
            # the new counts into the plan
            b.complete = False
        elif b.pending < 0:
            raise RuntimeError(
                "GradSync: a gradient event arrived after its bucket's all-reduce was launched (step "
                f"signature {self._sig!r} delivered more events than the learned plan); the all-reduce read a "
                "partial gradient")

    def _launch_ready(self):
        """The next-bucket rule: launch the run of complete buckets starting at the next index."""
        while self._next < len(self.buckets) and self.buckets[self._next].complete and \
                self.buckets[self._next].pending == 0 and self.buckets[self._next].expected > 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def _launch(self, b: _Bucket):
        if b.launched:
            return
        b.launched = True
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(ev)
                b.work = dist.all_reduce(self._wire(b), op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(self._wire(b), op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _wire(self, b: _Bucket):
        """The tensor the all-reduce moves: the bucket itself, or its bf16 copy (made on the current stream --
        the comm stream on the GPU -- into a buffer the bucket keeps)."""
        if self.comm_dtype == torch.float32:
            return b.buf
        if b.cbuf is None or b.cbuf.numel() != b.buf.numel():
            b.cbuf = torch.empty(b.buf.numel(), dtype=self.comm_dtype, device=b.buf.device)
        b.cbuf.copy_(b.buf)
        return b.cbuf

    def finish(self):
        """Join every bucket's all-reduce and average.  Call after backward, before the optimizer."""
        if not self._started:
            self._start_step()
        if self.buckets is None:
            self._build()  # first step: nothing overlapped yet
        if self._sig not in self.bucket_plans:
            self._learn(self._sig, self._seen)
        elif self._overlap:
            plan = self.plans[self._sig]
            if any(n > plan.get(i, 0) for i, n in self._seen.items()):
                # would have raised in _ready for a launched bucket; a bucket not yet launched is fine
                merged = dict(plan)
                for i, n in self._seen.items():
                    merged[i] = max(n, merged.get(i, 0))
                self._learn(self._sig, merged)
        if self.active:
            hooked = self._next
            for b in self.buckets[self._next:]:  # the rest, in index order
                self._launch(b)
            self._next = len(self.buckets)
            zero = [i for i, b in enumerate(self.buckets) if self._overlap and b.expected == 0]
            self.last_overlap = {"buckets": len(self.buckets), "from_hooks": hooked,
                                 "from_finish": len(self.buckets) - hooked, "overlap": self._overlap,
                                 "first_zero_plan_bucket": zero[0] if zero else None}
            if self._overlap:  # (a first sighting launches everything from finish() by design)
                self.left_to_finish[self._sig] = max(self.left_to_finish.get(self._sig, 0), len(self.buckets) - hooked)
            stats = self._launch_stats()
            for b in self.buckets:
                b.work.wait()
            if stats is not None:
                stats.wait()
            if self.cuda:
                torch.cuda.current_stream().wait_stream(self.comm)
            inv = 1.0 / self.world
            for b in self.buckets:
                if b.cbuf is not None and self.comm_dtype != torch.float32:
                    b.buf.copy_(b.cbuf)  # widen the reduced bf16 sum back into the fp32 gradients
                b.buf.mul_(inv)
            if stats is not None:
                self._stat_flat.mul_(inv)
                torch._foreach_copy_(self._stat_bufs, [v.view_as(t) for v, t in zip(
                    self._stat_flat.split([t.numel() for t in self._stat_bufs]), self._stat_bufs)])
        self._reset_step()

    def _launch_stats(self):
        """All-reduce (sum) of the BatchNorm running statistics, flattened, after the last bucket."""
        if not self._stat_bufs:
            return None
        n = sum(t.numel() for t in self._stat_bufs)
        if self._stat_flat is None or self._stat_flat.numel() != n:
            self._stat_flat = torch.empty(n, device=self._stat_bufs[0].device, dtype=torch.float32)
        torch.cat([t.reshape(-1).float() for t in self._stat_bufs], out=self._stat_flat)
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(ev)
                return dist.all_reduce(self._stat_flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return dist.all_reduce(self._stat_flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def remove(self):
        for h in self.hooks:
            h.remove()
        if self._listener in ops.GRAD_LISTENERS:
            ops.GRAD_LISTENERS.remove(self._listener)


def rank_cores(avail, slot: int, local_world: int):
    """The CPUs one local rank pins its process to: the slot-th of local_world contiguous, equal slices of the
    sorted usable CPUs (a contiguous slice keeps a rank on one socket when GPUs are numbered socket by socket);
    None when there are fewer CPUs than ranks (no pinning)."""
    avail = sorted(avail)
    per = len(avail) // max(int(local_world), 1)
    if per < 1 or not 0 <= slot < local_world:
        return None
    return avail[slot * per:(slot + 1) * per]


def broadcast_parameters(model: torch.nn.Module, src: int = 0):
    """Replicas start from rank 0's parameters and buffers."""
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)
