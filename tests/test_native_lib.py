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


def test_noise_uniform_never_hits_0_or_1():
    import numpy as np

    from oracle import noise

    # the extreme hash values map strictly inside (0, 1) in float32, so gumbel noise stays finite
    h = np.array([0, 0xFFFFFFFF], dtype=np.uint32)
    u = ((h >> np.uint32(9)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)
    assert u[0] > 0 and u[1] < 1
    g = noise.gumbel(12345, np.arange(1 << 20, dtype=np.uint64))
    assert np.all(np.isfinite(g))


def test_maxfactor_record_layout_and_grouping():
    """The numpy record the optimizer packs matches MFParam; rows pack 64 / gsz to a wave."""
    from asrx import lib, optim

    assert optim._REC.itemsize == lib.load().asrx_maxfactor_param_bytes() == 144
    assert [optim._group(n) for n in (1, 2, 3, 5, 15, 16, 17, 64, 65, 40000)] == [1, 2, 4, 8, 16, 16, 32, 64, 64, 64]


def test_attention_mode_switch():
    """fp8 attention is a forward-only mode layered on the bf16 perf mode."""
    import pytest

    from asrx import prec

    with prec.precision("bf16"):
        assert prec.attention_prec() == prec.PREC_BF16
        with prec.attention("fp8"):
            assert prec.attention_prec() == prec.PREC_FP8ATT
            with prec.precision("fp32"):  # parity mode ignores the attention mode
                assert prec.attention_prec() == prec.PREC_F32
        assert prec.attention_prec() == prec.PREC_BF16
    with pytest.raises(ValueError):
        prec.set_attention("fp16")


def test_keyed_noise_index_guards():
    """Sequences past 8192 positions (or streams x channels past the 32-bit index) would alias keyed
    noise draws: refused before any kernel runs."""
    import pytest

    from asrx import ops

    ops._noise_rows_ok(96, 1024, 3001)  # tiny/medium 30 s, B = 32 x 3 streams: fine
    with pytest.raises(ValueError, match="8192"):
        ops._noise_rows_ok(2, 384, 8193)
    with pytest.raises(ValueError, match="32-bit"):
        ops._noise_rows_ok(2000, 1024, 3001)


def test_msheath_plan_struct_layout():
    """The ctypes mirror of asrx_msheath_plan / asrx_msheath_layer (asrx/msheath.py) has the C structs' sizes and
    the workspace query runs on the host (no GPU): the composite no-save MSheath forward reads them by layout."""
    import ctypes

    from asrx import lib, msheath

    L = lib.load()
    assert L.asrx_msheath_plan_bytes() == ctypes.sizeof(msheath._Plan)
    assert L.asrx_msheath_layer_bytes() == ctypes.sizeof(msheath._Layer)
    layers = (msheath._Layer * 2)()
    for i in range(2):
        layers[i].M, layers[i].Dh = 64, 192
    plan = msheath._Plan(p_hidden=128, H1=1536, n_layers=2, layers=ctypes.addressof(layers))
    n = L.asrx_msheath_fwd_ws_bytes(ctypes.byref(plan), 2, 3001, 384)
    assert n > 4 * 2 * 3001 * 384 * 6  # at least the running x, px, out, hln, hh and SH rows
