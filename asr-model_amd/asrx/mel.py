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


FB_A, FB_B = 8, 24  # taps of a lane's two bands in the kernel (csrc/logmel.hip)


def lane_filterbank(fb: torch.Tensor):
    """Pack the filterbank for the log-mel kernel's lanes.

    Lane m of a wave owns two bands: band_a (the 64 lowest, <= FB_A taps) and band_b (<= FB_B
    taps), each read as even-aligned pairs of power bins starting at an even bin.  The two 32-lane
    halves of a wave read the power buffer in separate LDS cycles, so the bands are split between
    them such that few lanes of a half hit the same bank (bank = (start/2) mod 32 for 8-byte reads).
    Returns (ints[256] = band_a | band_b | start_a | start_b, weights[8, 64, 4] float32 holding
    w/4 — the kernel forms 4|X|^2)."""
    starts, w = sparse_filterbank(fb)
    n_mels = fb.shape[1]
    assert n_mels == 128
    width = (w > 0).sum(1)
    sp = [int(s) & ~1 for s in starts]

    def split(bands):
        groups, seen = [[], []], [{}, {}]
        for b in sorted(bands, key=lambda b: ((sp[b] // 2) % 32, sp[b])):
            r = (sp[b] // 2) % 32
            opts = [i for i in (0, 1) if len(groups[i]) < 32]
            i = min(opts, key=lambda i: (len(seen[i].get(r, set()) | {sp[b]}), len(groups[i])))
            groups[i].append(b)
            seen[i].setdefault(r, set()).add(sp[b])
        return groups[0] + groups[1]

    lanes_a, lanes_b = split(list(range(64))), split(list(range(64, 128)))
    ints = torch.zeros(256, dtype=torch.int32)
    wts = torch.zeros(FB_A + FB_B, 64, dtype=torch.float32)
    for lane in range(64):
        for slot, (band, taps, off) in enumerate(((lanes_a[lane], FB_A, 0), (lanes_b[lane], FB_B, FB_A))):
            s0, sh = sp[band], int(starts[band]) - sp[band]
            if int(width[band]) + sh > taps:
                raise ValueError(f"band {band} needs {int(width[band]) + sh} taps > {taps}")
            ints[slot * 64 + lane] = band
            ints[128 + slot * 64 + lane] = s0
            wts[off + sh: off + sh + int(width[band]), lane] = 0.25 * w[band, : int(width[band])]
    return ints, wts.view(8, 4, 64).permute(0, 2, 1).contiguous()


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
        ints, wts = lane_filterbank(mel_filterbank())
        _DEV_CACHE[key] = (fft_consts().to(device), wts.to(device), ints.to(device))
    return _DEV_CACHE[key]


def n_frames(n_samples: int) -> int:
    return 1 + n_samples // HOP


def algorithmic_bytes(B: int, N: int, pool: bool) -> float:
    """read N*4 + write 128*F*4 per clip (+ the pooled waveform feature)."""
    F = n_frames(N)
    return float(B * (N * 4 + N_MELS * F * 4 + ((N // HOP) * 4 if pool else 0)))


def algorithmic_flops(B: int, N: int) -> float:
    """fp32 flops of the log-mel per batch, counted for the textbook algorithm the kernel implements: per frame the
    Hann window (1024 mul), the 1024-point real FFT as a 512-point complex FFT (5 n log2 n = 23040) plus the real
    untangle (~10 per bin, 5120), the power (3 per bin, 1539), the 128-band HTK filterbank (one multiply-add per
    tap, every bin in at most two bands: 2052) and the log / scale (~3 per band): 33159 per frame.  At ~29 flop per
    algorithmic HBM byte the kernel sits right of the fp32 ridge (157 TF/s / 8 TB/s = 19.7 flop/B): its binding
    roofline is the fp32 vector rate, not HBM."""
    per_frame = 1024 + 5 * 512 * 9 + 10 * 512 + 3 * 513 + 2 * 1026 + 3 * N_MELS
    return float(B * n_frames(N) * per_frame)


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
    ws = torch.empty(lib.load().asrx_logmel_ws_bytes(B, N) // 4, dtype=torch.float32, device=wav.device)
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


def wave_pool(wav: torch.Tensor, T: int) -> torch.Tensor:
    """adaptive_avg_pool1d of (B, N) float32 device audio to T bins (essentials.py:493-510) for any N
    (asrx_wave_pool; logmel(pool=True) fuses the 160 | N case into the mel pass)."""
    lib.require_gpu(wav)
    if wav.dim() == 1:
        wav = wav.unsqueeze(0)
    if wav.dtype != torch.float32 or wav.stride(-1) != 1:
        raise ValueError("wave_pool expects float32 audio with unit inner stride")
    B, N = wav.shape
    out = torch.empty(B, T, device=wav.device, dtype=torch.float32)
    lib.call("asrx_wave_pool", lib.ptr(wav), B, N, wav.stride(0), T, lib.ptr(out), lib.stream())
    return out
