"""Synthetic LibriSpeech-shaped clips (SURVEY.md §8(d) "Synthetic inputs"): there is no dataset in
the image, so the benchmark and the tests generate seeded clips of the same shape."""
from __future__ import annotations

import numpy as np
import torch

SR = 16000


def waveform(n_clips: int, seconds: float = 30.0, first_seed: int = 1000) -> torch.Tensor:
    """(B, N) float32: 0.5 sin(2 pi f n/sr)(1 + 0.3 sin(2 pi 3 n/sr)) + 0.05 N(0,1), f ~ U[100, 300] Hz,
    seed 1000 + b, peak-normalised (the file branch of load_wave, essentials.py:310-312)."""
    n = int(seconds * SR)
    t = np.arange(n, dtype=np.float64) / SR
    out = np.empty((n_clips, n), dtype=np.float32)
    for b in range(n_clips):
        rng = np.random.default_rng(first_seed + b)
        f = rng.uniform(100.0, 300.0)
        x = 0.5 * np.sin(2 * np.pi * f * t) * (1 + 0.3 * np.sin(2 * np.pi * 3 * t)) + 0.05 * rng.standard_normal(n)
        out[b] = x / np.abs(x).max()
    return torch.from_numpy(out)


def pitch(n_clips: int, frames: int = 3001, first_seed: int = 1000, mask_seed: int = 2000) -> torch.Tensor:
    """(B, 1, frames) f0 track f_b (1 + 0.05 sin(2 pi t / 300)), 20 % unvoiced (zero) frames."""
    out = np.empty((n_clips, 1, frames), dtype=np.float32)
    t = np.arange(frames, dtype=np.float64)
    for b in range(n_clips):
        f = np.random.default_rng(first_seed + b).uniform(100.0, 300.0)
        voiced = np.random.default_rng(mask_seed + b).random(frames) >= 0.2
        out[b, 0] = (f * (1 + 0.05 * np.sin(2 * np.pi * t / 300.0))) * voiced
    return torch.from_numpy(out)


def text(n_clips: int, length: int = 256, vocab: int = 40000, seed: int = 7):
    """text_ids = [BOS] + U[3, vocab)^(length-1), labels = text_ids[:, 1:] ++ [EOS] (no padding)."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(3, vocab, (n_clips, length), generator=g, dtype=torch.int64)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((n_clips, 1), 2, dtype=torch.int64)], 1)
    return ids, labels
