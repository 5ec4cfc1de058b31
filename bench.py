#!/usr/bin/env python
"""Headline benchmark: audio-sec/sec fwd+bwd on 30 s / 16 kHz clips (BASELINE.json `metric`).

One step = the hot path over one batch of synthetic clips already resident in HBM:
  log-mel + waveform pool (HIP) on the raw 30 s waveforms -> Model.forward (tiny config,
  BASELINE configs[1]: 4 enc / 4 dec, d=384, 6 heads, bf16 MFMA) -> cross entropy -> backward ->
  (N > 1) RCCL bucketed gradient all-reduce overlapped with backward, joined before the step ends.
Weak scaling: every rank processes its own B clips; `value` is the whole-job aggregate.

python bench.py --gpus N --steps K --warmup W         (N > 1: launched by torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CLIP_SECONDS = 30.0
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFS = 2500.0   # dense bf16 MFMA (spec, no sparsity)
F32_PEAK_TFS = 157.3     # fp32 MFMA == fp32 vector peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--batch", type=int, default=32, help="clips per GPU")
    ap.add_argument("--text-len", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "x3"],
                    help="bf16: the perf mode (headline); fp32: exact fp32 MFMA (parity); x3: fp32 storage with "
                         "split-bf16 GEMM products and fp32 attention (the gradient mode that follows the reference)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the live per-kernel event probe")
    ap.add_argument("--no-optimizer", action="store_true", help="skip timing the fused MaxFactor step")
    ap.add_argument("--dist-backend", default="nccl", help="process-group backend for N > 1 (nccl = RCCL); "
                    "gloo + --same-device is a one-GPU rehearsal of the multi-rank path")
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0 (rehearsal only)")
    ap.add_argument("--graph", action="store_true", help="N=1 only: capture the step in one HIP graph and replay it "
                    "(measured 5 %% SLOWER than eager launches: the replay runs the side streams' kernels mostly one "
                    "at a time, profiles/r05_eager_vs_graph.txt)")
    ap.add_argument("--eager", action="store_true", help="eager launches (the default; kept for old scripts)")
    ap.add_argument("--dist-single", action="store_true", help="N=1 through the N>1 code path: a 1-rank "
                    "process group (RCCL) and GradSync's bucket all-reduces on the comm stream (a rehearsal of "
                    "the multi-GPU step on a one-GPU box; never the headline)")
    ap.add_argument("--pitch-frames", type=int, default=3001, help="pitch stream length of the timed step "
                    "(3001: SURVEY.md §8(d)'s synthetic spec, = the spectrogram's frames)")
    ap.add_argument("--no-refpitch-line", action="store_true", help="skip the side line at the reference's own "
                    "pitch shape (6001 frames: pw.dio's 5 ms frames, essentials.py:451-455)")
    ap.add_argument("--dead-at", default=None, choices=["start", "mid", "end"], help="where the dead blocks' side-stream "
                    "work is enqueued (asrx.model.processor.dead_blocks_at; default: the model's)")
    ap.add_argument("--graph-dead", action="store_true", help="replay the dead blocks from HIP graphs "
                    "(asrx.model.processor.graph_dead_blocks; off by default, profiles/r06_host_vs_gpu.txt)")
    ap.add_argument("--no-pin", action="store_true", help="N > 1: do not pin each rank to its own slice of the CPUs")
    ap.add_argument("--bucket-mb", type=float, default=64.0, help="N > 1: GradSync bucket size in MB (the first bucket "
                    "a quarter of it)")
    ap.add_argument("--bf16-grads", action="store_true", help="N > 1: all-reduce the gradient buckets in bf16 "
                    "(asrx.dist.GradSync comm_dtype; opt-in, fp32 by default)")
    ap.add_argument("--no-fp32-line", action="store_true", help="skip the side lines in the fp32 and x3 parity "
                    "modes (same workload; the modes that meet north_star's parity gate)")
    ap.add_argument("--fp32-steps", type=int, default=3)
    ap.add_argument("--no-dead-block-line", action="store_true", help="skip the extra measurement with the "
                    "reference's dead decoder blocks eliminated (reported beside, never as, the headline)")
    return ap.parse_args()


def cpu_baseline(model, cfg_name, warmup=1, runs=3):
    """The oracle (op-for-op CPU restatement of the reference forward, fp32) timed on the host cores on a
    bounded sample of the same workload: one 30 s clip through mel + forward + backward at the same
    config, `warmup` untimed runs then the median of `runs` (warm-ups + median; a
    30 s tiny clip costs ~5 s of CPU per run, so 1 + 3 keeps the sample near 20 s)."""
    import statistics

    import numpy as np

    from asrx import synth
    from asrx.config import CONFIGS
    from oracle import mel as omel
    from oracle import model as om

    cfg = CONFIGS[cfg_name]
    P = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    for k, v in P.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
            v.requires_grad_(True)
    wav = synth.waveform(1, CLIP_SECONDS)
    pitch = synth.pitch(1)
    ids, labels = synth.text(1)
    times = []
    for i in range(warmup + runs):
        for v in P.values():
            v.grad = None
        t0 = time.perf_counter()
        spec = torch.from_numpy(omel.log_mel(wav[0].numpy().astype(np.float64))).float().unsqueeze(0)
        wf = torch.from_numpy(omel.waveform_feature(wav[0].numpy())).float().unsqueeze(0)
        out = om.forward(P, {"dims": cfg.dims, "head": cfg.head, "layer": cfg.layer}, ids, labels,
                         spectrogram=spec, pitch=pitch, waveform=wf, seed=0, step=i, dtype=torch.float32)
        out["loss"].backward()
        if i >= warmup:
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": CLIP_SECONDS / med, "unit": "audio-sec/sec", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"1 x 30 s clip, {cfg_name} config, T=256, oracle mel + fwd + bwd, fp32, batch 1: "
                      f"{warmup} warm-up + median of {runs} ({med:.2f} s per clip)"}


def plumbing_line(dev, warmup=3, runs=10):
    """BASELINE configs[0]: one 1 s clip -> log-mel (128, 101) -> 2-layer D=256 AudioEncoder forward
    (model.py:120-169, eval), on the CPU oracle (the reference's CPU plumbing case, fp32) and on the HIP
    path (fp32 parity mode, the same chain) -- 3 warm-ups + the median of 10 each."""
    import statistics

    import numpy as np

    from asrx import prec
    from asrx.config import CONFIGS
    from asrx.mel import logmel
    from asrx.model import AudioEncoder
    from asrx.noise import NoiseCtx
    from oracle import mel as omel
    from oracle import model as om

    c = CONFIGS["plumbing"]
    torch.manual_seed(0)
    enc = AudioEncoder(c.mels, c.dims, c.head, c.layer, c.act, c.n_type).eval()
    P = {"enc." + k: v.detach().clone() for k, v in enc.state_dict().items()}
    g = np.random.default_rng(5)
    audio = (0.5 * np.sin(2 * np.pi * 220.0 * np.arange(16000) / 16000) + 0.05 * g.standard_normal(16000))
    audio = (audio / np.abs(audio).max()).astype(np.float32)

    def cpu():
        with torch.no_grad():
            spec = torch.from_numpy(omel.log_mel(audio.astype(np.float64))).float().unsqueeze(0)
            return om.encode_stream(P, spec, c.layer, om.Noise(0, 0, torch.float32), [0], training=False)

    tc = []
    for i in range(warmup + runs):
        t0 = time.perf_counter()
        ref = cpu()
        if i >= warmup:
            tc.append(time.perf_counter() - t0)
    enc = enc.to(dev)
    wav = torch.from_numpy(audio).to(dev).view(1, -1)
    tg = []
    with prec.precision("fp32"), torch.no_grad():
        for i in range(warmup + runs):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = enc.layers(enc.stem(logmel(wav, layout="BMF")), NoiseCtx(0, 0, False), 0)
            torch.cuda.synchronize()
            if i >= warmup:
                tg.append(time.perf_counter() - t0)
    err = float((out.double().cpu() - ref.double()).abs().max() / ref.double().abs().max())
    return {"workload": "BASELINE configs[0]: 1 x 1 s clip -> log-mel (128, 101) -> 2-layer d=256 encoder forward",
            "cpu_oracle_ms": round(statistics.median(tc) * 1e3, 3), "cpu_threads": torch.get_num_threads(),
            "hip_fp32_ms": round(statistics.median(tg) * 1e3, 3),
            "hip_vs_oracle_max_rel": err, "timing": f"{warmup} warm-ups + median of {runs}",
            "shape": list(out.shape)}


def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n):
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run (one process per
    GPU, rendezvous on 127.0.0.1) as a child and exit with its status.  Runs before anything touches
    the GPU (this process never initialises HIP), so no exec or fork happens after GPU init."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # stdout carries exactly one JSON line: everything else written to fd 1 from here on -- the RCCL version banner
    # of communicator init, library messages, our own progress prints -- goes to stderr, and the line is written to
    # the original stdout at the end
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.same_device:
        local = 0
    # one issue thread per rank: pin each rank's process (its Python issue thread and the HIP runtime's threads) to its
    # own contiguous slice of the CPUs this job may use, before anything touches the GPU, so eight ranks' host
    # issue does not migrate across each other's cores (local ranks map to GPUs in order, and contiguous core
    # slices keep a rank on one socket when the GPUs are numbered socket by socket)
    cores = None
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1 and not args.no_pin and hasattr(os, "sched_setaffinity"):
        from asrx.dist import rank_cores  # (no GPU touched by the import)
        cores = rank_cores(os.sched_getaffinity(0), int(os.environ.get("LOCAL_RANK", "0")), local_world)
        if cores:
            os.sched_setaffinity(0, cores)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.dist_single
    if args.dist_single and world == 1 and "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    if distributed:
        if args.dist_backend == "nccl":
            # no device_id: RCCL's communicator is then created at the first collective (the parameter broadcast)
            # on the device set above.  The eager form (device_id=dev) measured 12 ms slower per tiny step in
            # every later step, with or without collectives in them -- 1-rank group, 192.5 vs 180.5 ms, the
            # lazy form at the N = 1 step time (profiles/r06_rccl_eager_init_ab.txt)
            dist.init_process_group("nccl")
        else:
            dist.init_process_group(args.dist_backend)

    from asrx import prec, probe, synth
    from asrx.config import CONFIGS
    from asrx.dist import GradSync, broadcast_parameters
    from asrx.mel import algorithmic_bytes, algorithmic_flops, logmel
    from asrx.model import Model

    prec.set_precision(args.precision)
    cfg = CONFIGS[args.config]
    torch.manual_seed(0)
    model = Model(cfg).to(dev).train()
    if args.dead_at:
        model.processor.dead_blocks_at = args.dead_at
    model.processor.graph_dead_blocks = args.graph_dead
    if distributed:
        broadcast_parameters(model)
    gsync = GradSync(model, bucket_mb=args.bucket_mb, reduce_single=args.dist_single,
                     comm_dtype=torch.bfloat16 if args.bf16_grads else torch.float32)
    model.set_noise(seed=0, step=rank * 1_000_000)

    B = args.batch
    wav = synth.waveform(B, CLIP_SECONDS, first_seed=1000 + rank * B).to(dev)
    pitch = synth.pitch(B, frames=args.pitch_frames, first_seed=1000 + rank * B, mask_seed=2000 + rank * B).to(dev)
    ids, labels = synth.text(B, args.text_len, cfg.tokens, seed=7 + rank)
    ids, labels = ids.to(dev), labels.to(dev)

    def step():
        gsync.zero_grad()
        # the kernel writes (B, F, 128) (what the encoder's k3 conv consumes); the model receives the
        # reference's (B, 128, F) spectrogram as a transposed view of it, so no copy is made
        spec, wfeat = logmel(wav, layout="BFM", pool=True)
        out = model(labels=labels, text_ids=ids, spectrogram=spec.transpose(1, 2), pitch=pitch,
                    waveform=wfeat.unsqueeze(1))
        out["loss"].backward()
        gsync.finish()
        return out["loss"]

    # eager launches at every N: the N = 1 point of a 1 -> 8 curve runs the same code path as N > 1, and
    # eager is the faster one (profiles/r05_eager_vs_graph.txt)
    use_graph = args.graph and not args.eager and not distributed
    # warm-up on the stream the timed steps run on: the caching allocator keeps freed blocks per stream, so a
    # warm-up on another stream leaves the first timed steps to allocate (hipMalloc) their whole working set --
    # ~0.7 s per step of a 3-step medium run (profiles/r06_host_vs_gpu.txt).  A graph capture needs its warm-up
    # off the default stream, and then captures and replays there too.
    side = torch.cuda.Stream() if use_graph else torch.cuda.current_stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(max(args.warmup, 1 if use_graph else 0)):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = None
    if use_graph:
        # One training step -> one HIP graph: every launch (kernels, memsets, events of the probe) is
        # recorded once and replayed, so the host cost per step is one graphLaunch.  All control
        # flow of the step is on device (masked MSheath, no host syncs), so the replay is the step.
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            loss = step()
        torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    from asrx import lib
    host_s = 0.0  # host time spent issuing the steps (eager: Python + launches); ~ms_per_step means host-bound
    for i in range(args.steps):
        h0 = time.perf_counter()
        if graph is not None:
            # the captured launches carry the capture step's noise keys: a new epoch per replay gives
            # every timed step its own dropout masks and gumbel draws (stream-ordered, outside the graph)
            lib.call("asrx_set_noise_epoch", i + 1, lib.stream())
            graph.replay()
        else:
            loss = step()
        host_s += time.perf_counter() - h0
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if graph is not None:
        lib.call("asrx_set_noise_epoch", 0, lib.stream())
    # host_issue_ms_per_step above includes the time the host spends BLOCKED in launches once the GPU's queues are
    # full, so it approaches ms_per_step whenever the GPU is the bound too.  Issue time without that back-pressure:
    # steps started from an idle GPU (synchronised before each), the host's own time to issue one step, beside
    # that step's wall time -- issue well below wall means the step is GPU-bound (profiles/r06_host_vs_gpu.txt)
    free_issue, free_wall = [], []
    if graph is None:
        for _ in range(2):
            torch.cuda.synchronize()
            h0 = time.perf_counter()
            step()
            h1 = time.perf_counter()
            torch.cuda.synchronize()
            free_issue.append(h1 - h0)
            free_wall.append(time.perf_counter() - h0)
    if not args.no_probe:
        # per-kernel HIP events stay out of the timed region (and cannot be read back from inside a
        # captured graph): every rank runs the identical step (same kernels, shapes and inputs)
        # once more eagerly with the probe on, right after the timed steps
        probe.enable(("gemm", "logmel", "attn"))
        # per-kernel event times without concurrent streams
        model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = False
        step()
        model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = True
        torch.cuda.synchronize()
        recs = probe.disable()
        probe_steps = 1
    else:
        recs = None
    opt_ms = None
    if not args.no_optimizer:
        # the reference's MaxFactor step (model.py:772-787 groups and
        # hyper-parameters) as one fused native call over every parameter with a gradient; timed
        # after the measured steps, not part of `value` (the metric is fwd + bwd)
        from asrx.optim import MaxFactor, reference_param_groups
        opt = MaxFactor(reference_param_groups(model), lr=2.5e-3, b_decay=-0.8, eps=(1e-8, 1e-8), d=1.0,
                        decay=1e-2, gamma=0.99, max=False, bias=1, min_lr=1e-9, clip=False, cap=0.0)
        opt.step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            opt.step()
        e1.record()
        torch.cuda.synchronize()
        opt_ms = e0.elapsed_time(e1) / 5
    if distributed:
        # replicas must hold identical averaged gradients after the all-reduce
        gsum = torch.stack([p.grad.double().norm() for p in model.parameters() if p.grad is not None]).sum()
        lo, hi = gsum.clone(), gsum.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        grad_spread = float((hi - lo) / hi.clamp_min(1e-30))
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        core_map = [None] * world
        dist.all_gather_object(core_map, None if cores is None else f"{cores[0]}-{cores[-1]}" if cores == list(
            range(cores[0], cores[-1] + 1)) else ",".join(map(str, cores)))
    loss_v = float(loss.item())

    audio_s = world * B * CLIP_SECONDS * args.steps
    value = audio_s / elapsed
    result = {
        "metric": "audio-sec/sec fwd+bwd on 30s@16kHz LibriSpeech-shaped clips (whole job, all GPUs)",
        "value": round(value, 3),
        "unit": "audio-sec/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (SURVEY.md §8(d) seeded clips, random-init weights)",
        "config": {"workload": f"{args.config}{' (BASELINE configs[1])' if args.config == 'tiny' else ''}: log-mel + "
                               f"{cfg.layer} enc/{cfg.layer} dec d={cfg.dims} h={cfg.head} fwd+bwd, {B} x 30 s clips "
                               f"per GPU, T={args.text_len}",
                   "model": args.config, "global_batch": world * B, "seq_len": 3001, "text_len": args.text_len,
                   "pitch_frames": args.pitch_frames,
                   "parallelism": f"dp{world}"},
        "per_gpu": round(value / world, 3),
        "host_issue_ms_per_step": round(host_s / args.steps * 1e3, 3),
        **({"host_issue_from_idle_ms": round(min(free_issue) * 1e3, 3),
            "step_from_idle_ms": round(min(free_wall) * 1e3, 3),
            "host_issue_note": "host_issue_ms_per_step includes launches blocked on full GPU queues; "
                               "host_issue_from_idle_ms is one step issued from an idle GPU (min of 2) beside that "
                               "step's wall time step_from_idle_ms: issue < wall means the GPU is the bound"}
           if free_issue else {}),
        **({"grad_sync_rel_spread": grad_spread, "cpu_affinity_by_rank": core_map,
            "grad_wire_dtype": "bf16" if args.bf16_grads else "fp32"} if distributed else {}),
        **({"dist_single": "1-rank RCCL group through the N>1 path (eager, bucket all-reduces on the comm "
                           "stream); a rehearsal, not the headline"} if args.dist_single else {}),
        "loss": loss_v,
    }
    if recs is not None:
        n, _, sec = probe.summarize(recs["gemm"])
        flops = sum(probe.gemm_flops(tag, w) for w, _, _, tag in recs["gemm"])
        # x3: a split-bf16 product costs three bf16 MFMAs, so its GEMM ceiling is a third of the bf16 peak in
        # useful (fp32-equivalent) flops; its attention runs the fp32 kernels
        peak = {"bf16": BF16_PEAK_TFS, "fp32": F32_PEAK_TFS, "x3": BF16_PEAK_TFS / 3}[args.precision]
        apeak = {"bf16": BF16_PEAK_TFS, "fp32": F32_PEAK_TFS, "x3": F32_PEAK_TFS}[args.precision]
        achieved = flops / sec / 1e12 if sec > 0 else 0.0
        step_s = elapsed / args.steps
        # dominant kernel: gemm_wr_kernel, the wide bf16-weight GEMM behind every activation x weight product of
        # the forward and of the input gradients -- EVERY instantiation (plain, MSheath row-list, residual,
        # tied logits + CE statistics, AbbyNormal router, activation-gradient), i.e. the same launch set as the
        # rocprof summary's gemm_wr_kernel rows and the PMC table's `traffic`.  At K, N <= 1536 its arithmetic
        # intensity is below the MI355X ridge (2500 TF/s / 8 TB/s = 312 flop/B), so its roofline is HBM
        # bandwidth; algorithmic bytes per launch: probe.gemm_wr_bytes (row-list launches use the tile count
        # the device built, read back after the probed step)
        wn_n, wn_bytes, wn_flops, wn_sec, unknown = 0, 0.0, 0.0, 0.0, 0
        for w, e0, e1, tag in recs["gemm"]:
            byts = probe.gemm_wr_bytes(tag)
            if byts is None:
                unknown += int(bool(tag) and tag[0] == "wn")
                continue
            wn_n += 1
            wn_bytes += byts
            wn_flops += probe.gemm_flops(tag, w)
            wn_sec += e0.elapsed_time(e1) * 1e-3
        probe.clear_aux()
        if wn_sec > 0:
            gbs = wn_bytes / wn_sec / 1e9
            result["roofline"] = {"kernel": "asrx::wn::gemm_wr_kernel + gemm_p2_kernel + gemm_ws_kernel + "
                                            "router64_kernel, every instantiation (the wide bf16-weight MFMA GEMM: "
                                            "plain, row-list, residual, rotary, tied logits, router, "
                                            "activation-gradient; gemm_p2 = its two-workgroups-per-CU form, gemm_ws = "
                                            "its weight-stationary form, router64 = the d = 64 router launches)",
                                  "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(gbs / HBM_PEAK_GBS, 4),
                                  **pmc_traffic(("gemm_wr_kernel", "gemm_p2_kernel", "gemm_ws_kernel", "router64_kernel"),
                                                args.config,
                                                args.batch, args.pitch_frames),
                                  "algorithmic_bytes_per_launch": round(wn_bytes / wn_n),
                                  "algorithmic_bytes_per_step": round(wn_bytes / probe_steps),
                                  "launches_per_step": wn_n // probe_steps,
                                  **({"launches_unaccounted": unknown} if unknown else {}),
                                  "avg_us": round(wn_sec / wn_n * 1e6, 2),
                                  "share_of_step": round(wn_sec / probe_steps / step_s, 3),
                                  "mfma_achieved_tflops": round(wn_flops / wn_sec / 1e12, 2),
                                  "mfma_frac": round(wn_flops / wn_sec / 1e12 / peak, 4),
                                  "recompute": "frac = algorithmic_bytes_per_step / (gemm_wr_kernel + gemm_p2_kernel + "
                                               "gemm_ws_kernel + router64_kernel time per step in the rocprof summary) "
                                               "/ peak"}
        result["gemm_all"] = {"kernel": "every asrx GEMM launch (wide, generic fp32/bf16 incl. wgrad, router)",
                              "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                              "frac": round(achieved / peak, 4),
                              "launches_per_step": n // probe_steps,
                              "avg_us": round(sec / max(n, 1) * 1e6, 2),
                              "share_of_step": round(sec / probe_steps / step_s, 3)}
        n2, byts, sec2 = probe.summarize(recs["logmel"])
        if sec2 > 0:
            gbs = byts / sec2 / 1e9
            mfl = algorithmic_flops(B, wav.shape[1]) * n2  # one probe record per asrx_logmel call
            result["mel_roofline"] = {"kernel": "asrx_logmel (frames + finalize)", "bound": "hbm",
                                      "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": round(gbs / HBM_PEAK_GBS, 4),
                                      "algorithmic_bytes": algorithmic_bytes(B, wav.shape[1], True),
                                      "avg_us": round(sec2 / n2 * 1e6, 1),
                                      # the same launches against the fp32 vector roofline (the binding one:
                                      # 33 kflop per 1.15 KB frame, right of the ridge; asrx.mel.algorithmic_flops)
                                      "valu_achieved_tflops": round(mfl / sec2 / 1e12, 2), "valu_peak": F32_PEAK_TFS,
                                      "valu_frac": round(mfl / sec2 / 1e12 / F32_PEAK_TFS, 4),
                                      "algorithmic_flops": algorithmic_flops(B, wav.shape[1])}
        n3, af, sec3 = probe.summarize(recs["attn"])
        if sec3 > 0:
            result["attn_fwd"] = {"achieved": round(af / sec3 / 1e12, 2), "unit": "TFLOP/s", "peak": apeak,
                                  "frac": round(af / sec3 / 1e12 / apeak, 4),
                                  "share_of_step": round(sec3 / probe_steps / step_s, 3)}
    if opt_ms is not None:
        result["maxfactor_step_ms"] = round(opt_ms, 3)
    result["launch"] = "hip-graph replay" if graph is not None else "eager"
    if recs is not None:
        result["probe"] = "per-kernel HIP events on one eager pass of the same step after the timed steps"
    if not args.no_dead_block_line and not distributed:
        # SURVEY.md §7 "Only the last block reaches the output": processor.forward computes blocks
        # 0..L-2 and discards them.  The headline keeps that work (faithful); this line measures the
        # same step with them skipped (output-identical under keyed noise), labelled as such.
        model.processor.skip_dead_blocks = True
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        g2 = None
        if graph is not None:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            if g2 is not None:
                lib.call("asrx_set_noise_epoch", i + 1, lib.stream())
                g2.replay()
            else:
                step()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t1
        if g2 is not None:
            lib.call("asrx_set_noise_epoch", 0, lib.stream())
        model.processor.skip_dead_blocks = False
        result["dead_block_eliminated"] = {
            "value": round(B * CLIP_SECONDS * args.steps / el2, 3), "unit": "audio-sec/sec",
            "ms_per_step": round(el2 / args.steps * 1e3, 3),
            "note": "same step with processor blocks 0..L-2 skipped (they never reach the output, model.py:617-628); "
                    "output-identical, NOT the headline"}
    if not args.no_refpitch_line and not distributed and args.pitch_frames != 6001:
        # VERDICT r02 "missing 3": the step the reference's own feature path produces.  extract_features
        # calls pw.dio(x, sr, frame_period) (essentials.py:451-455), which binds frame_period to f0_floor and
        # keeps dio's 5 ms frames: a 30 s clip yields a 6001-frame pitch stream beside the 3001-frame
        # spectrogram, so the three audio streams no longer share one batched pass and the pitch stream
        # runs a 6001^2 self-attention.  Same model, clips and text; reported beside the headline.
        pitch_keep = pitch  # step() reads `pitch` from this scope
        pitch = synth.pitch(B, frames=6001, first_seed=1000 + rank * B, mask_seed=2000 + rank * B).to(dev)
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        g3 = None
        if graph is not None:
            g3 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g3):
                step()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for i in range(args.steps):
            if g3 is not None:
                lib.call("asrx_set_noise_epoch", i + 1, lib.stream())
                g3.replay()
            else:
                step()
        torch.cuda.synchronize()
        el3 = time.perf_counter() - t2
        if g3 is not None:
            lib.call("asrx_set_noise_epoch", 0, lib.stream())
        del g3
        pitch = pitch_keep
        result["refpitch_workload"] = {
            "value": round(B * CLIP_SECONDS * args.steps / el3, 3), "unit": "audio-sec/sec",
            "ms_per_step": round(el3 / args.steps * 1e3, 3), "pitch_frames": 6001, "spectrogram_frames": 3001,
            "note": "reference extract_args workload: pitch at dio's 5 ms frames (essentials.py:451-455), "
                    "the step the reference's own feature path produces; NOT the headline (SURVEY.md §8(d) "
                    "specifies 3001-frame pitch)"}
    def mode_line(mode, steps, note):
        """The same workload in another precision mode (asrx.prec), timed here so the driver observes it, with its
        GEMMs priced against that mode's MFMA ceiling (fp32: the fp32 MFMA peak; x3: a third of the bf16 peak in
        fp32-equivalent flops) and its attention forward against the fp32 peak (both modes run fp32 attention)."""
        prec.set_precision(mode)
        try:
            step()  # warm-up: fp32 storage allocates a different working set
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            el4 = time.perf_counter() - t4
            line = {"value": round(B * CLIP_SECONDS * steps / el4, 3), "unit": "audio-sec/sec",
                    "ms_per_step": round(el4 / steps * 1e3, 3), "steps": steps, "warmup": 1, "dtype": mode,
                    "note": note}
            if not args.no_probe:
                probe.enable(("gemm", "attn"))
                model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = False
                step()
                model.processor.concurrent_dead_text = model.processor.concurrent_dead_blocks = True
                torch.cuda.synchronize()
                r4 = probe.disable()
                n4, _, s4 = probe.summarize(r4["gemm"])
                fl4 = sum(probe.gemm_flops(tag, w) for w, _, _, tag in r4["gemm"])
                probe.clear_aux()
                gpeak = {"fp32": F32_PEAK_TFS, "x3": BF16_PEAK_TFS / 3}[mode]
                if s4 > 0:
                    line["gemm_all"] = {"bound": "mfma", "achieved": round(fl4 / s4 / 1e12, 2), "peak": round(gpeak, 1),
                                        "unit": "TFLOP/s", "frac": round(fl4 / s4 / 1e12 / gpeak, 4),
                                        "launches_per_step": n4, "share_of_step": round(s4 / (el4 / steps), 3)}
                na, fa, sa = probe.summarize(r4["attn"])
                if sa > 0:
                    line["attn_fwd"] = {"achieved": round(fa / sa / 1e12, 2), "unit": "TFLOP/s", "peak": F32_PEAK_TFS,
                                        "frac": round(fa / sa / 1e12 / F32_PEAK_TFS, 4)}
            return line
        finally:
            prec.set_precision(args.precision)

    if not args.no_fp32_line and not distributed and args.precision == "bf16":
        # the parity modes on the same config, batch and clips, driver-observed.  fp32 (exact
        # fp32 MFMA) and x3 (split-bf16 GEMM products, fp32 attention) both meet north_star's parity gate: argmax ids
        # bit-exact and logits within max(1e-3, 30x the reference's own fp32 error) of the float64 oracle
        # (tests/test_gpu_model_configs.py; measured values in profiles/r06_parity_metrics.jsonl)
        result["fp32_workload"] = mode_line("fp32", args.fp32_steps, "same workload in the fp32 parity mode (exact "
                                            "fp32 MFMA, fp32 storage); NOT the headline")
        result["x3_workload"] = mode_line("x3", args.fp32_steps, "same workload in the x3 mode (fp32 storage, GEMM "
                                          "products as three bf16 MFMAs of hi / lo splits, fp32 attention): argmax "
                                          "bit-exact like fp32 mode; NOT the headline")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(model, args.config)
        result["configs0_plumbing"] = plumbing_line(dev)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(result) + "\n").encode())
    os.close(json_fd)


def pmc_traffic(kernel_substrs, config, batch, pitch_frames):
    """HBM bytes per launch of a kernel from the newest committed PMC table OF THIS WORKLOAD (profiles/
    rNN_pmc_traffic_<config>_b<batch>_p<pitch frames>_vM.csv: separate rocprofv3 FETCH_SIZE and WRITE_SIZE
    passes over one eager step of `bench.py --config C --batch B --no-refpitch-line --no-dead-block-line`,
    FETCH doubled per the gfx950 note, see tools/pmc_traffic.py), launch-weighted over every template
    instance whose name contains one of kernel_substrs.  PMC counters cannot be read inside the timed run, so the
    figure comes from the profiling pass of the same step; null when no table of this workload exists."""
    import csv
    import glob
    pat = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                       f"r*_pmc_traffic_{config}_b{batch}_p{pitch_frames}_v*.csv")
    key = lambda p: tuple(int(v) for v in re.search(r"r(\d+)_pmc_traffic_.*_v(\d+)\.csv$", p).groups())  # noqa: E731
    tabs = sorted(glob.glob(pat), key=key)
    if not tabs:
        return {"traffic": None, "traffic_note": f"no PMC table for {config} B={batch} pitch {pitch_frames}"}
    n, tot = 0, 0.0
    for r in csv.DictReader(open(tabs[-1])):
        if any(k in r["kernel"] for k in kernel_substrs):
            n += int(r["launches"])
            tot += int(r["launches"]) * float(r["avg_hbm_bytes"])
    if n == 0:
        return {"traffic": None}
    return {"traffic": round(tot / n), "traffic_unit": "B/launch",
            "traffic_source": os.path.join("profiles", os.path.basename(tabs[-1]))}


if __name__ == "__main__":
    main()
