"""Keyed noise sites for the reference's randomness (gumbel_softmax at essentials.py:170 and
model.py:476; nn.Dropout at model.py:107, 147).

A site key is FNV-1a-32 of "{seed}/{step}/{site}"; the device kernels hash (key, logical index)
(csrc/common.h).  Sample ids: text rows use b; audio stream s (a=pitch 0, b=spectrogram 1,
c=waveform 2) uses s*B + b.  The oracle restates this independently (oracle/keys.py).
"""
from __future__ import annotations

LSTRIDE = 8192


def site_key(seed: int, step: int, site: str) -> int:
    h = 0x811C9DC5
    for byte in f"{seed}/{step}/{site}".encode():
        h ^= byte
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


class NoiseCtx:
    def __init__(self, seed: int, step: int, training: bool):
        self.seed, self.step, self.training = seed, step, training

    def key(self, site: str) -> int:
        return site_key(self.seed, self.step, site)
