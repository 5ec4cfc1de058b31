"""Regenerate the golden fixtures in this directory from the oracle (oracle/): a 1 s log-mel +
waveform-feature vector, BASELINE configs[0]'s plumbing encoding of that clip (D=256, 2 layers), and a
toy-model forward (D=128, H=2, layer=4, V=1000, B=2, T=8, S=101).
The reference itself cannot be executed here, so these vectors pin the oracle
restatement against regressions; parity with the reference is unpinned.

    python tests/golden/make_golden.py            (all)
    python tests/golden/make_golden.py plumbing   (plumbing_1s.safetensors only)
"""
import os
import sys

import numpy as np
import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]

def pinned_threads():
    """One BLAS / torch intra-op thread while making or checking a fixture: the float64 oracle's reductions
    (matmul, FFT filterbank) are then summed in one order on every host -- with the host's default thread
    count the toy model's logits moved by ~1e-6 relative between an 8- and a 16-CPU container (its hard
    decisions amplify reduction-order ulps), which no rtol-1e-9 pin can absorb."""
    import contextlib

    from threadpoolctl import threadpool_limits

    @contextlib.contextmanager
    def ctx():
        n = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            with threadpool_limits(1):
                yield
        finally:
            torch.set_num_threads(n)

    return ctx()


TOY = dict(tokens=1000, mels=128, dims=128, head=2, layer=4, act="gelu", n_type="AbbyNormal")


def toy_inputs():
    g = torch.Generator().manual_seed(1)
    B, T, S, V = 2, 8, 101, 1000
    spec = torch.randn(B, 128, S, generator=g)
    pitch = torch.rand(B, 1, S, generator=g) * 200
    wav = torch.randn(B, 1, S - 1, generator=g) * 0.1
    ids = torch.randint(3, V, (B, T), generator=g)
    ids[:, 0] = 1
    labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1)
    labels[1, -2:] = 0
    return spec, pitch, wav, ids, labels


def toy_params():
    from asrx.config import Dimensions
    from asrx.model import Model

    torch.manual_seed(0)
    m = Model(Dimensions(**TOY))
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def param_checksum(P):
    return torch.tensor([float(sum(v.double().sum() for k, v in sorted(P.items()) if v.is_floating_point()))],
                        dtype=torch.float64)


def plumbing_params():
    """BASELINE configs[0]'s encoder (asrx CONFIGS['plumbing']: D=256, 2 layers) at seed 0, reference names."""
    from asrx.config import CONFIGS
    from asrx.model import AudioEncoder

    c = CONFIGS["plumbing"]
    torch.manual_seed(0)
    enc = AudioEncoder(c.mels, c.dims, c.head, c.layer, c.act, c.n_type)
    return {"enc." + k: v.detach().clone() for k, v in enc.state_dict().items()}


def plumbing_encoding(audio):
    """configs[0]: 1 s clip -> float64 oracle log-mel (128, 101) -> 2-layer D=256 AudioEncoder forward (eval)
    -> (1, 101, 256) (model.py:149-163)."""
    from oracle import mel as omel
    from oracle import model as om

    spec = torch.from_numpy(omel.log_mel(np.asarray(audio, dtype=np.float64))).unsqueeze(0)
    P = {k: v.double() if v.is_floating_point() else v for k, v in plumbing_params().items()}
    return om.encode_stream(P, spec, 2, om.Noise(0, 0, torch.float64), [0], training=False)


def write_plumbing():
    from safetensors.torch import load_file

    audio = load_file(os.path.join(HERE, "mel_1s.safetensors"))["audio"].numpy()
    save_file({"encoding": plumbing_encoding(audio).contiguous(), "param_checksum": param_checksum(plumbing_params())},
              os.path.join(HERE, "plumbing_1s.safetensors"))


def main():
    from oracle import mel as omel
    from oracle import model as om

    rng = np.random.default_rng(42)
    t = np.arange(16000) / 16000.0
    audio = (0.6 * np.sin(2 * np.pi * 440.0 * t) + 0.05 * rng.standard_normal(16000)).astype(np.float32)
    save_file({"audio": torch.from_numpy(audio),
               "logmel": torch.from_numpy(omel.log_mel(audio.astype(np.float64))),
               "waveform": torch.from_numpy(omel.waveform_feature(audio.astype(np.float64)))},
              os.path.join(HERE, "mel_1s.safetensors"))
    write_plumbing()

    spec, pitch, wav, ids, labels = toy_inputs()
    P = toy_params()
    Pd = {k: v.double() if v.is_floating_point() else v for k, v in P.items()}
    out = {}
    for name, training in (("train", True), ("eval", False)):
        r = om.forward(Pd, {"dims": 128, "head": 2, "layer": 4}, ids, labels, spectrogram=spec, pitch=pitch,
                       waveform=wav, seed=7, step=3, training=training)
        out[f"logits_{name}"] = r["logits"].detach()
        out[f"loss_{name}"] = r["loss"].detach().reshape(1)
    save_file({"spectrogram": spec, "pitch": pitch, "waveform": wav, "text_ids": ids, "labels": labels,
               "param_checksum": param_checksum(P), **out}, os.path.join(HERE, "toy_model.safetensors"))
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    with pinned_threads():
        if sys.argv[1:] == ["plumbing"]:
            write_plumbing()
        else:
            main()
