"""The C-ABI library loads (no GPU needed) and exports every symbol include/asrx.h declares."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "asrx.h")).read()
    return sorted(set(re.findall(r"\b(asrx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from asrx import lib

    L = lib.load()
    syms = header_symbols()
    assert len(syms) >= 5
    for s in syms:
        assert hasattr(L, s), s
    # the Python binding declares a signature for every header entry point and nothing else
    assert sorted(lib.SIGNATURES) == syms


def test_abi_version_and_error_channel():
    from asrx import lib

    L = lib.load()
    assert L.asrx_abi_version() >= 1
    assert isinstance(L.asrx_last_error(), bytes)


def test_noise_hash_matches_oracle():
    from asrx import lib
    from oracle import noise

    L = lib.load()
    rng = np.random.default_rng(0)
    keys = rng.integers(0, 2**32, 8, dtype=np.uint64)
    idx = rng.integers(0, 2**32, 64, dtype=np.uint64)
    for k in keys:
        ours = noise.hash32(int(k), idx)
        for i, h in zip(idx, ours):
            assert L.asrx_noise_hash(int(k), int(i)) == int(h)


def test_mel_frames():
    from asrx import lib

    L = lib.load()
    assert L.asrx_mel_frames(480000) == 3001
    assert L.asrx_mel_frames(16000) == 101
