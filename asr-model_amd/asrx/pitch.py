"""GPU pitch: pyworld.dio + pyworld.stonemask, as extract_features calls them.

essentials.py:451-455 runs, per clip on the CPU,
    f0, t = pw.dio(x, sample_rate, frame_period)        # 3rd positional = f0_floor (quirk)
    f0 = pw.stonemask(x, f0, t, sample_rate)
This module runs a batch of equal-length clips on the device in float64 (csrc/pitch.hip): the same
DIO stages (50 Hz low-cut, per-band Nuttall low-pass, four zero-crossing interval series per band
interpolated to the frame times, best band per frame, FixF0Contour) and StoneMask's instantaneous-
frequency refinement.  The API mirrors pyworld's: dio(x, fs, f0_floor, f0_ceil, channels_in_octave,
frame_period, speed, allowed_range) -> (f0, t) and stonemask(x, f0, t, fs) -> f0, on numpy arrays or
torch tensors ((N,) or (B, N)); reference_pitch(audio) is the extract_features call as written.
pyworld / WORLD are absent here: parity is against the float64 restatement oracle/pitch.py, and is
**unpinned** against pyworld itself.  speed != 1 (decimation) is not built.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import lib

CUTOFF_HZ = 50.0
_TAPS: dict = {}


def _mround(x):
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def _plan(fs, f0_floor, f0_ceil, channels_in_octave, device):
    """Filter taps and band table for one (fs, f0 range) on the device (cached)."""
    key = (fs, f0_floor, f0_ceil, channels_in_octave, str(device))
    if key in _TAPS:
        return _TAPS[key]
    nb = 1 + int(math.log(f0_ceil / f0_floor) / math.log(2.0) * channels_in_octave)
    bf0 = np.array([f0_floor * 2.0 ** ((i + 1) / channels_in_octave) for i in range(nb)], dtype=np.float64)
    # zero-phase low-cut: taps -c..c of delta minus a normalised raised-cosine low-pass of N = 2c + 1
    N = _mround(fs / CUTOFF_HZ) * 2 + 1
    c = (N - 1) // 2
    w = 0.5 - 0.5 * np.cos(np.arange(1, N + 1) * 2.0 * math.pi / (N + 1))
    lc = -w / w.sum()
    lc[c] += 1.0
    # Nuttall low-pass of 4 round(fs / f0_b / 2) taps per band
    wins, offs, lens, off = [], [], [], 0
    for b in bf0:
        n = 4 * _mround(fs / b / 2.0)
        t = np.arange(n) / (n - 1.0)
        wins.append(0.355768 - 0.487396 * np.cos(2 * math.pi * t) + 0.144232 * np.cos(4 * math.pi * t)
                    - 0.012604 * np.cos(6 * math.pi * t))
        offs.append(off)
        lens.append(n)
        off += n
    plan = dict(nb=nb, bf0=bf0, c=c, lc=torch.from_numpy(lc).to(device),
                nut=torch.from_numpy(np.concatenate(wins)).to(device),
                offs=np.array(offs, dtype=np.int64), lens=np.array(lens, dtype=np.int64))
    _TAPS[key] = plan
    return plan


def _as_batch(x, device):
    """(B, N) float32 on the device from an (N,) / (B, N) numpy array or tensor; flag for 1-D input."""
    one = False
    if not torch.is_tensor(x):
        x = torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if x.dim() == 1:
        x, one = x.unsqueeze(0), True
    x = x.to(device=device, dtype=torch.float32)
    if not x.is_contiguous():
        x = x.contiguous()
    return x, one


def _device(x):
    if torch.is_tensor(x) and x.is_cuda:
        return x.device
    return torch.device("cuda")


def dio(x, fs, f0_floor=71.0, f0_ceil=800.0, channels_in_octave=2.0, frame_period=5.0, speed=1,
        allowed_range=0.1):
    """pyworld.dio on the GPU.  x: (N,) or (B, N) (numpy or tensor; float64 input is computed from
    its float32 rounding, the reference passes float32 audio cast to float64).  Returns (f0 float64
    (B, F) or (F,), temporal_positions float64 (F,)) as tensors on the device."""
    if speed != 1:
        raise NotImplementedError("dio: speed != 1 (decimation) is not built (the reference uses 1)")
    dev = _device(x)
    xb, one = _as_batch(x, dev)
    lib.require_gpu(xb)
    B, N = xb.shape
    p = _plan(float(fs), float(f0_floor), float(f0_ceil), float(channels_in_octave), dev)
    F = int(1000.0 * N / fs / frame_period) + 1
    ylen = N + 1
    cap = max(ylen // 4, 4)
    E = lambda *s: torch.empty(*s, dtype=torch.float64, device=dev)  # noqa: E731
    mean, hp, f = E(B), E(B, ylen + 2 * p["c"]), E(B, ylen)
    ev, cand, score, work, f0 = E(B, 4, cap), E(B, p["nb"], F), E(B, p["nb"], F), E(B, 3 * F), E(B, F)
    offs = p["offs"].ctypes.data_as(ctypes.c_void_p)
    lens = p["lens"].ctypes.data_as(ctypes.c_void_p)
    bf0 = p["bf0"].ctypes.data_as(ctypes.c_void_p)
    lib.call("asrx_pitch_dio", lib.ptr(xb), xb.stride(0), B, N, float(fs), float(f0_floor), float(f0_ceil),
             float(frame_period), float(allowed_range), lib.ptr(p["lc"]), p["c"], lib.ptr(p["nut"]), offs, lens, bf0,
             p["nb"], lib.ptr(mean), lib.ptr(hp), lib.ptr(f), lib.ptr(ev), cap, lib.ptr(cand), lib.ptr(score),
             lib.ptr(work), lib.ptr(f0), F, lib.stream())
    t = torch.arange(F, dtype=torch.float64, device=dev) * frame_period / 1000.0
    return (f0[0] if one else f0), t


def stonemask(x, f0, temporal_positions, fs):
    """pyworld.stonemask on the GPU for the frames of dio (uniform temporal positions)."""
    dev = _device(x)
    xb, one = _as_batch(x, dev)
    B, N = xb.shape
    f0 = torch.as_tensor(f0, dtype=torch.float64, device=dev)
    f0 = f0.reshape(B, -1).contiguous()
    t = torch.as_tensor(temporal_positions, dtype=torch.float64)
    F = f0.shape[1]
    fp = float(t[1] - t[0]) * 1000.0 if F > 1 else 5.0
    if F > 1 and not torch.allclose(t.cpu(), torch.arange(F, dtype=torch.float64) * fp / 1000.0):
        raise ValueError("stonemask: temporal positions must be dio's uniform frame times")
    out = torch.empty(B, F, dtype=torch.float64, device=dev)
    lib.call("asrx_pitch_stonemask", lib.ptr(xb), xb.stride(0), B, N, float(fs), lib.ptr(f0), fp, F, lib.ptr(out),
             lib.stream())
    return out[0] if one else out


def reference_pitch(audio, sample_rate=16000, hop_length=160):
    """extract_features' pitch (essentials.py:451-455) as written: dio(x, fs, frame_period) binds
    frame_period to f0_floor, so f0_floor = hop / sr * 1000 and frames are 5 ms."""
    frame_period = hop_length / sample_rate * 1000
    f0, t = dio(audio, sample_rate, frame_period)
    return stonemask(audio, f0, t, sample_rate)
