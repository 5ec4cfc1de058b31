"""Keyed counter-based noise, restated bit-for-bit from csrc/common.h (mix32 / noise_uniform).

The reference draws fresh torch RNG inside F.gumbel_softmax (essentials.py:170, model.py:476) and
nn.Dropout (model.py:107, 147).  For parity both the HIP path and this oracle take the same draws,
addressed by (site key, logical element index) so that batching or evaluation order cannot change
which sample gets which noise.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def hash32(key: int, idx):
    key = np.uint64(key & 0xFFFFFFFF)
    k1 = (key * np.uint64(0x9E3779B9) + np.uint64(0x632BE5AB)) & M32
    return (_mix32((_mix32(np.asarray(idx, dtype=np.uint64) ^ key) + k1) & M32)).astype(np.uint32)


def uniform(key: int, idx):
    """u in [2^-24, 1 - 2^-24]: ((h >> 9) + 0.5) / 2^23, computed in float32 like the device."""
    h = hash32(key, idx)
    return ((h >> np.uint32(9)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)


def gumbel(key: int, idx):
    """Gumbel(0,1) = -log(E), E = -log(u) ~ Exp(1) (torch: -exponential_().log())."""
    u = uniform(key, idx).astype(np.float32)
    return -np.log(-np.log(u))
