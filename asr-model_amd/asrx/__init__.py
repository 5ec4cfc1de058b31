"""asrx — MI355X-native hot path of the sine2pi/ASR-model speech recogniser.

Public surface mirroring the reference: `Dimensions`, `Model` (model.py), `extract_features`,
`DataCollator` (essentials.py).  Compute runs in libasrx.so (HIP, gfx950) via the C-ABI.
"""
from .config import CONFIGS, Dimensions  # noqa: F401

__all__ = ["Dimensions", "CONFIGS"]
