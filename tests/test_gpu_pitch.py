"""GPU pitch (asrx/pitch.py, csrc/pitch.hip) against the float64 restatement oracle/pitch.py on the
same clips: dio f0 (voicing decisions and values), stonemask (same input f0), and the reference's
extract_features call (f0_floor bound to the frame period, 5 ms frames) at the bench's 30 s shape.
The GPU filters by direct convolution where the oracle (like WORLD) multiplies FFT spectra: values
agree to float64 rounding, so a decision may flip only on an exact tie."""
import numpy as np
import pytest
import torch

from oracle import pitch as P

pytestmark = pytest.mark.gpu
FS = 16000


def _clips(seconds=1.5):
    n = int(FS * seconds)
    t = np.arange(n) / FS
    rng = np.random.default_rng(3)
    a = sum(0.5 / k * np.sin(2 * np.pi * 120 * k * t) for k in range(1, 5))
    f = 220 * (1 + 0.05 * np.sin(2 * np.pi * 3 * t))  # vibrato
    b = 0.4 * np.sin(2 * np.pi * np.cumsum(f) / FS) + 0.1 * np.sin(4 * np.pi * np.cumsum(f) / FS)
    c = a.copy()
    c[n // 3:n // 2] = 0.0  # unvoiced gap
    c[n // 2:] = 0.3 * rng.standard_normal(n - n // 2)  # noise
    x = np.stack([a, b, c]) + 1e-3 * rng.standard_normal((3, n))
    return x.astype(np.float32)


def _agree(g, r):
    g, r = np.asarray(g, dtype=np.float64), np.asarray(r, dtype=np.float64)
    same_voicing = ((g > 0) == (r > 0)).mean()
    both = (g > 0) & (r > 0)
    rel = np.abs(g[both] - r[both]) / r[both] if both.any() else np.zeros(1)
    return same_voicing, (rel < 1e-6).mean() if both.any() else 1.0


def test_dio_matches_oracle(cuda):
    from asrx import pitch

    x = _clips()
    f0, t = pitch.dio(torch.from_numpy(x).cuda(), FS, 71.0, 800.0, 2.0, 5.0)
    f0 = f0.cpu().numpy()
    assert f0.shape == (3, int(1000.0 * x.shape[1] / FS / 5.0) + 1)
    for i in range(3):
        r, tr = P.dio(x[i].astype(np.float64), FS, 71.0, 800.0, 2.0, 5.0)
        assert np.allclose(t.cpu().numpy(), tr)
        sv, close = _agree(f0[i], r)
        assert sv >= 0.99 and close >= 0.99, (i, sv, close)
    assert (f0[0] > 0).mean() > 0.95 and abs(np.median(f0[0][f0[0] > 0]) / 120 - 1) < 5e-3


def test_stonemask_matches_oracle(cuda):
    from asrx import pitch

    x = _clips()
    for i in range(3):
        f, t = P.dio(x[i].astype(np.float64), FS)
        r = P.stonemask(x[i].astype(np.float64), f, t, FS)
        g = pitch.stonemask(torch.from_numpy(x[i]).cuda(), f, t, FS).cpu().numpy()
        v = r > 0
        assert np.array_equal(g > 0, v)
        assert np.abs(g[v] - r[v]).max() / r[v].max() < 1e-8


def test_reference_pitch_30s_clip(cuda):
    """extract_features' call at the bench clip length: 30 s -> 6001 frames (5 ms, f0_floor 10 Hz)."""
    from asrx import pitch, synth

    x = synth.waveform(1, 30.0)[0].numpy()
    g = pitch.reference_pitch(torch.from_numpy(x).cuda()).cpu().numpy()
    r = P.reference_pitch(x)
    assert g.shape == r.shape == (6001,)
    sv, close = _agree(g, r)
    assert sv >= 0.99 and close >= 0.99, (sv, close)


def test_extract_features_pitch_and_phase(cuda):
    from asrx.features import extract_features

    class Tok:
        def encode(self, s):
            return [5]

    x = _clips(2.0)[0]
    out = extract_features({"audio": {"array": x, "sampling_rate": FS}, "sentence": "a"}, tokenizer=Tok(),
                           pitch=True, phase=True)
    assert out["pitch"].shape == (1, int(1000.0 * len(x) / FS / 5.0) + 1) and out["pitch"].is_cuda
    assert out["phase"].shape == (int(1000.0 * len(x) / FS / 10.0) + 1,)
    f0 = out["pitch"][0].cpu().numpy()
    assert abs(np.median(f0[f0 > 0]) / 120 - 1) < 1e-3
    ph = out["phase"].cpu().numpy()
    assert ph.min() >= 0 and ph.max() < 2 * np.pi
