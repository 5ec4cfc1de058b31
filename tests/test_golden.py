"""Golden fixtures (tests/golden/, made by make_golden.py from the oracle): the CPU suite pins the
oracle against them; the GPU suite checks the HIP path against the stored vectors."""
import os
import sys

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def test_oracle_reproduces_mel_golden():
    from oracle import mel as omel

    g = load_file(os.path.join(HERE, "mel_1s.safetensors"))
    audio = g["audio"].numpy().astype(np.float64)
    with mg.pinned_threads():
        assert np.array_equal(omel.log_mel(audio), g["logmel"].numpy())
        assert np.array_equal(omel.waveform_feature(audio), g["waveform"].numpy())


def test_oracle_reproduces_toy_model_golden():
    from oracle import model as om

    g = load_file(os.path.join(HERE, "toy_model.safetensors"))
    P = mg.toy_params()
    assert torch.allclose(mg.param_checksum(P), g["param_checksum"], rtol=1e-12), "Model init changed"
    Pd = {k: v.double() if v.is_floating_point() else v for k, v in P.items()}
    with mg.pinned_threads():
        r = om.forward(Pd, {"dims": 128, "head": 2, "layer": 4}, g["text_ids"], g["labels"],
                       spectrogram=g["spectrogram"], pitch=g["pitch"], waveform=g["waveform"], seed=7, step=3,
                       training=True)
    assert torch.allclose(r["logits"], g["logits_train"], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["train", "eval"])
def test_hip_model_matches_golden(cuda, mode):
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model

    g = load_file(os.path.join(HERE, "toy_model.safetensors"))
    torch.manual_seed(0)
    model = Model(Dimensions(**mg.TOY)).to(cuda).train(mode == "train")
    model.set_noise(7, 3)
    with prec.precision("fp32"), torch.no_grad():
        out = model(labels=g["labels"].to(cuda), text_ids=g["text_ids"].to(cuda),
                    spectrogram=g["spectrogram"].to(cuda), pitch=g["pitch"].to(cuda), waveform=g["waveform"].to(cuda))
    lg, lr = out["logits"].double().cpu(), g[f"logits_{mode}"]
    assert float((lg - lr).abs().max() / lr.abs().max()) < 1e-3
    assert torch.equal(lg.argmax(-1), lr.argmax(-1))
    assert abs(float(out["loss"]) - float(g[f"loss_{mode}"])) / abs(float(g[f"loss_{mode}"])) < 1e-3


@pytest.mark.gpu
def test_hip_mel_matches_golden(cuda):
    from asrx.mel import logmel

    g = load_file(os.path.join(HERE, "mel_1s.safetensors"))
    s, w = logmel(g["audio"].view(1, -1).to(cuda), layout="BMF", pool=True)
    assert float((s[0].double().cpu() - g["logmel"]).abs().max()) < 2e-4
    assert float((w.double().cpu() - g["waveform"]).abs().max()) < 1e-6
