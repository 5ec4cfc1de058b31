"""float64 numpy restatement of the reference's spectrogram + waveform features.

essentials.py:469-491 — torchaudio MelSpectrogram(sample_rate=16000, n_fft=1024, hop_length=160,
f_min=50, f_max=8000, n_mels=128, window_fn=torch.hann_window, center=True, pad_mode="constant",
power=2.0, mel_scale="htk", norm=None, normalized=False) then clamp(min=1e-10).log10(),
maximum(x, x.max() - 8), (x + 4) / 4.  torchaudio is absent; its documented
algorithm is restated: torch.stft(center=True) zero-pads n_fft//2 on both sides, frames at hop
160 -> 1 + N//160 frames, periodic Hann, one-sided |rFFT|^2, then spec^T @ fb with the triangular
HTK filterbank (melscale_fbanks, norm=None).

essentials.py:493-510 — waveform feature: adaptive_avg_pool1d(audio, int(N/16000*100)).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
from __future__ import annotations

import math

import numpy as np

N_FFT, HOP, N_MELS, SR, F_MIN, F_MAX = 1024, 160, 128, 16000, 50.0, 8000.0


def hz_to_mel(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_to_hz(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def filterbank(n_freqs=N_FFT // 2 + 1, f_min=F_MIN, f_max=F_MAX, n_mels=N_MELS, sr=SR):
    """(n_freqs, n_mels) float64 triangular HTK filterbank (torchaudio melscale_fbanks, norm=None)."""
    all_freqs = np.linspace(0.0, sr // 2, n_freqs)
    f_pts = mel_to_hz(np.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2))
    f_diff = np.diff(f_pts)
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def hann_periodic(n=N_FFT):
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)


def power_spectrogram(audio):
    """(n_freqs, F) |STFT|^2 with center=True zero padding (torch.stft semantics)."""
    x = np.asarray(audio, dtype=np.float64)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="constant")
    n_frames = 1 + (len(xp) - N_FFT) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    frames = xp[idx] * hann_periodic()[None, :]
    spec = np.fft.rfft(frames, axis=1)
    return (np.abs(spec) ** 2).T


def log_mel(audio):
    """(128, F) float64 spectrogram feature exactly as essentials.py:486-490 computes it."""
    mel = filterbank().T @ power_spectrogram(audio)
    log_m = np.log10(np.maximum(mel, 1e-10))
    log_m = np.maximum(log_m, log_m.max() - 8.0)
    return (log_m + 4.0) / 4.0


def waveform_feature(audio, sample_rate=SR, hop_length=HOP):
    """(1, T) adaptive_avg_pool1d of the clip to int(N/sr * sr/hop) frames (essentials.py:494-503)."""
    x = np.asarray(audio, dtype=np.float64)
    n = len(x)
    target = int((n / sample_rate) * (sample_rate // hop_length))
    out = np.empty(target)
    for i in range(target):  # torch adaptive pool bins: [floor(i*n/T), ceil((i+1)*n/T))
        s = (i * n) // target
        e = -((-(i + 1) * n) // target)
        out[i] = x[s:e].mean()
    return out[None, :]
