"""BASELINE configs[0] ("single 1 s @16 kHz random clip -> log-mel + 2-layer/d=256 encoder forward on CPU
reference (plumbing, no GPU)"): 1 s clip -> log-mel (128, 101) -> AudioEncoder(D=256, 2 layers) forward
(model.py:120-169, eval) -> (1, 101, 256).  The CPU part pins the oracle against the committed fixture
(tests/golden/plumbing_1s.safetensors, tests/golden/make_golden.py); the GPU part runs the same chain
through the HIP log-mel and encoder."""
import os
import sys

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def _golden():
    return load_file(os.path.join(HERE, "plumbing_1s.safetensors")), load_file(os.path.join(HERE, "mel_1s.safetensors"))


def test_oracle_reproduces_plumbing_golden():
    g, m = _golden()
    assert torch.allclose(mg.param_checksum(mg.plumbing_params()), g["param_checksum"], rtol=1e-12), "init changed"
    with mg.pinned_threads():
        enc = mg.plumbing_encoding(m["audio"].numpy())
    assert enc.shape == (1, 101, 256)
    assert torch.equal(enc, g["encoding"])


def _hip_encoder(cuda):
    from asrx.config import CONFIGS
    from asrx.model import AudioEncoder

    c = CONFIGS["plumbing"]
    torch.manual_seed(0)
    return AudioEncoder(c.mels, c.dims, c.head, c.layer, c.act, c.n_type).to(cuda).eval()


def run_hip_plumbing(enc, audio=None, spec=None):
    """audio (N,) on the device -> HIP log-mel (or a given (1, 128, F) spec) -> HIP encoder (1, F, D)."""
    from asrx.mel import logmel
    from asrx.noise import NoiseCtx

    if spec is None:
        spec = logmel(audio.view(1, -1), layout="BMF")  # (1, 128, F)
    with torch.no_grad():
        return enc.layers(enc.stem(spec), NoiseCtx(0, 0, False), 0)


@pytest.mark.gpu
@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 3e-2)])
@pytest.mark.parametrize("chain", ["oracle_mel", "hip_mel"])
def test_hip_plumbing_matches_golden(cuda, precision, tol, chain):
    """oracle_mel: the HIP encoder on the fixture's float64 log-mel; hip_mel: the whole chain from the
    waveform (the HIP log-mel's ~1e-4 rounding on top: 10x the encoder tolerance in fp32)."""
    from asrx import prec

    g, m = _golden()
    enc = _hip_encoder(cuda)
    with prec.precision(precision):
        if chain == "hip_mel":
            out = run_hip_plumbing(enc, audio=m["audio"].to(cuda))
            tol = tol * 10 if precision == "fp32" else tol
        else:
            out = run_hip_plumbing(enc, spec=m["logmel"].float().unsqueeze(0).to(cuda))
    ref = g["encoding"]
    assert out.shape == ref.shape
    err = float((out.double().cpu() - ref).abs().max() / ref.abs().max())
    print(precision, "plumbing encoder max rel err", err)
    assert err < tol, err
