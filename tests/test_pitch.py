"""Pitch oracle (oracle/pitch.py: float64 restatement of pyworld dio + stonemask as extract_features
calls them, essentials.py:451-455) pinned by known-answer tests -- pyworld / WORLD are absent, so its
parity with pyworld itself is unpinned.  CPU only."""
import numpy as np
import pytest

from oracle import pitch as P

FS = 16000


def _tone(f0, seconds=1.5, harmonics=4, noise=1e-3, seed=0):
    t = np.arange(int(FS * seconds)) / FS
    x = sum(0.5 / k * np.sin(2 * np.pi * f0 * k * t + 0.3 * k) for k in range(1, harmonics + 1))
    return x + noise * np.random.default_rng(seed).standard_normal(len(t))


@pytest.mark.parametrize("f0", [90.0, 155.0, 240.0, 410.0])
def test_dio_stonemask_known_f0(f0):
    x = _tone(f0)
    f, t = P.dio(x, FS, 71.0, 800.0, 2.0, 5.0)
    assert len(f) == len(t) == int(1000.0 * len(x) / FS / 5.0) + 1
    assert np.allclose(t, np.arange(len(t)) * 0.005)
    v = f > 0
    assert v.mean() > 0.95
    assert abs(np.median(f[v]) / f0 - 1) < 5e-3
    r = P.stonemask(x, f, t, FS)
    assert abs(np.median(r[v]) / f0 - 1) < 1e-3  # instantaneous-frequency refinement is tighter
    assert np.all(r[~v] == 0)


def test_silence_and_noise_are_unvoiced():
    assert P.reference_pitch(np.zeros(FS)).max() == 0.0
    noise = np.random.default_rng(1).standard_normal(FS) * 0.3
    f, _ = P.dio(noise, FS)
    assert (f > 0).mean() < 0.2


def test_reference_call_binds_frame_period_to_f0_floor():
    """essentials.py:452-454: pw.dio(x, sr, frame_period) -> f0_floor = 10 Hz, default 5 ms frames."""
    x = _tone(130.0, seconds=2.0)
    ref = P.reference_pitch(x.astype(np.float32), 16000, 160)
    f, t = P.dio(x.astype(np.float32).astype(np.float64), FS, 10.0, 800.0, 2.0, 5.0)
    assert len(ref) == int(1000.0 * len(x) / FS / 5.0) + 1  # 5 ms frames, not the 10 ms hop
    assert np.array_equal(ref, P.stonemask(x.astype(np.float32).astype(np.float64), f, t, FS))
    v = ref > 0
    assert v.mean() > 0.9 and abs(np.median(ref[v]) / 130.0 - 1) < 1e-3


def test_interp1_matches_matlab_semantics():
    x = np.array([0.0, 1.0, 2.0, 4.0])
    y = np.array([0.0, 10.0, 20.0, 0.0])
    xi = np.array([-1.0, 0.0, 0.5, 1.0, 3.0, 4.0, 5.0])
    assert np.allclose(P.interp1(x, y, xi), [-10.0, 0.0, 5.0, 10.0, 10.0, 0.0, -10.0])
