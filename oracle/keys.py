"""Noise-site naming shared (by convention, not by import) with asrx/noise.py.

A site key is FNV-1a-32 of "{seed}/{step}/{site}".  Row noise of an AbbyNormal call uses logical
index ((sid * H + h) * 8192 + l) * 3 + k, where sid is the sample id (text: b; audio stream s:
s * B + b), h the head (H = 1 for feature-wide norms), l the position; MSheath's policy gumbel
uses (sid * 64 + i) * 3 + k for layer i; dropout uses (sid * C + c) * 8192 + t.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
from __future__ import annotations

LSTRIDE = 8192


def site_key(seed: int, step: int, site: str) -> int:
    h = 0x811C9DC5
    for byte in f"{seed}/{step}/{site}".encode():
        h ^= byte
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h
