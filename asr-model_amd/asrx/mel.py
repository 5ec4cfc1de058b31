"""Log-mel front end (HIP kernel ``asrx_logmel``), replacing essentials.py:469-491 and the waveform
pool of essentials.py:493-510.

The filterbank is the torchaudio ``melscale_fbanks`` algorithm (HTK mel scale, ``norm=None``) as
documented for torchaudio: bins ``linspace(0, sr//2, n_fft//2+1)``, ``n_mels+2`` points equally
spaced in mel between ``f_min`` and ``f_max``, triangular filters
``max(0, min(-(slope_left)/Δleft, slope_right/Δright))``, all in float32 like the library.
torchaudio is not installed here; the restatement is pinned by the known-answer tests in
``tests/test_oracle.py`` (parity otherwise unpinned).
"""
from __future__ import annotations

import math

import torch

from . import lib, probe

N_FFT = 1024
HOP = 160
N_MELS = 128
F_MIN = 50.0
F_MAX = 8000.0
SAMPLE_RATE = 16000
FB_WIDTH = 32  # max nonzero bins per band kept by the kernel


def hz_to_mel_htk(f: float) -> float:
    return 2595.0 * math.log10(1.0 + f / 700.0)


def mel_filterbank(n_freqs: int = N_FFT // 2 + 1, f_min: float = F_MIN, f_max: float = F_MAX,
                   n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE,
                   dtype=torch.float32) -> torch.Tensor:
    """(n_freqs, n_mels) triangular HTK filterbank, norm=None."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs, dtype=dtype)
    m_pts = torch.linspace(hz_to_mel_htk(f_min), hz_to_mel_htk(f_max), n_mels + 2, dtype=dtype)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.minimum(down, up), min=0.0)


def sparse_filterbank(fb: torch.Tensor, width: int = FB_WIDTH):
    """Pack each band's contiguous nonzero bins: (start[n_mels] int32, weights[n_mels, width])."""
    n_freqs, n_mels = fb.shape
    starts = torch.zeros(n_mels, dtype=torch.int32)
    w = torch.zeros(n_mels, width, dtype=torch.float32)
    for m in range(n_mels):
        nz = torch.nonzero(fb[:, m] > 0).flatten()
        if nz.numel() == 0:
            continue
        s, e = int(nz[0]), int(nz[-1]) + 1
        if e - s > width:
            raise ValueError(f"band {m} spans {e - s} bins > {width}")
        starts[m] = s
        w[m, : e - s] = fb[s:e, m].float()
    return starts, w


def fft_consts(dtype=torch.float32) -> torch.Tensor:
    """window[1024] | tw512 (re,im)[512] | tw1024 (re,im)[513], float32."""
    win = torch.hann_window(N_FFT, periodic=True, dtype=torch.float32)
    m = torch.arange(512, dtype=torch.float64)
    a512 = -2.0 * math.pi * m / 512.0
    tw512 = torch.stack([torch.cos(a512), torch.sin(a512)], 1).flatten().float()
    k = torch.arange(513, dtype=torch.float64)
    a1024 = -2.0 * math.pi * k / 1024.0
    tw1024 = torch.stack([torch.cos(a1024), torch.sin(a1024)], 1).flatten().float()
    return torch.cat([win, tw512, tw1024])


_DEV_CACHE: dict = {}


def device_consts(device):
    key = str(device)
    if key not in _DEV_CACHE:
        starts, w = sparse_filterbank(mel_filterbank())
        _DEV_CACHE[key] = (fft_consts().to(device), w.contiguous().to(device),
                           starts.contiguous().to(device))
    return _DEV_CACHE[key]


def n_frames(n_samples: int) -> int:
    return 1 + n_samples // HOP


def algorithmic_bytes(B: int, N: int, pool: bool) -> float:
    """read N*4 + write 128*F*4 per clip (+ the pooled waveform feature)."""
    F = n_frames(N)
    return float(B * (N * 4 + N_MELS * F * 4 + ((N // HOP) * 4 if pool else 0)))


def logmel(wav: torch.Tensor, layout: str = "BFM", pool: bool = False):
    """Batched log-mel of (B, N) float32 device audio.

    layout "BMF" -> (B, 128, F) like the reference's (128, F) per clip; "BFM" -> (B, F, 128)
    (channels-last, what the encoder consumes).  With pool=True also returns the (B, N//160)
    waveform feature (adaptive_avg_pool1d to N/160 frames, essentials.py:495-503).
    """
    lib.require_gpu(wav)
    if wav.dim() == 1:
        wav = wav.unsqueeze(0)
    if wav.dtype != torch.float32 or wav.stride(-1) != 1:
        raise ValueError("logmel expects float32 audio with unit inner stride")
    B, N = wav.shape
    F = n_frames(N)
    consts, fbw, fbs = device_consts(wav.device)
    if layout == "BFM":
        out = torch.empty(B, F, N_MELS, device=wav.device, dtype=torch.float32)
        lay = 0
    elif layout == "BMF":
        out = torch.empty(B, N_MELS, F, device=wav.device, dtype=torch.float32)
        lay = 1
    else:
        raise ValueError(layout)
    ws = torch.empty(B, dtype=torch.int32, device=wav.device)
    pooled = None
    T = 0
    if pool:
        T = N // HOP
        if T * HOP != N:
            raise ValueError("fused waveform pool needs N to be a multiple of 160")
        pooled = torch.empty(B, T, device=wav.device, dtype=torch.float32)
    e0 = probe.begin("logmel")
    lib.call("asrx_logmel", lib.ptr(wav), B, N, wav.stride(0), lib.ptr(consts), lib.ptr(fbw),
             lib.ptr(fbs), lib.ptr(out), lay, F * N_MELS, lib.ptr(ws), lib.ptr(pooled), T, lib.stream())
    probe.end("logmel", e0, algorithmic_bytes(B, N, pool))
    return (out, pooled) if pool else out
