"""Model configuration — the reference's `Dimensions` (model.py:30-38), same fields and meaning."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class Dimensions:
    tokens: int
    mels: int
    dims: int
    head: int
    layer: int
    act: str
    n_type: str


# D/H/L per config (H chosen so that head_dim == 64); V = 40000 (tokenizer.json).
CONFIGS = {
    "plumbing": Dimensions(tokens=40000, mels=128, dims=256, head=4, layer=2, act="gelu", n_type="AbbyNormal"),
    "tiny": Dimensions(tokens=40000, mels=128, dims=384, head=6, layer=4, act="gelu", n_type="AbbyNormal"),
    "small": Dimensions(tokens=40000, mels=128, dims=768, head=12, layer=12, act="gelu", n_type="AbbyNormal"),
    "medium": Dimensions(tokens=40000, mels=128, dims=1024, head=16, layer=24, act="gelu", n_type="AbbyNormal"),
    # the reference's own main() configuration (model.py:746)
    "reference_main": Dimensions(tokens=40000, mels=128, dims=512, head=4, layer=4, act="gelu", n_type="AbbyNormal"),
}
