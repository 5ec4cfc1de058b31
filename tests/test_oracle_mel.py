"""Known-answer tests pinning the mel/waveform oracle (oracle/mel.py) and the host filterbank
(asrx/mel.py).  The reference has no tests of its own; these KATs come from
SURVEY.md §8(c)."""
import math

import numpy as np
import torch

from oracle import mel as omel


def test_frame_count():
    for n in (16000, 480000, 1, 159, 160, 161):
        assert omel.power_spectrogram(np.zeros(n)).shape[1] == 1 + n // 160


def test_silence_floor():
    # mel 0 -> clamp 1e-10 -> log10 = -10 everywhere -> max-8 clip inactive -> (-10+4)/4 = -1.5
    out = omel.log_mel(np.zeros(16000))
    assert out.shape == (128, 101)
    assert np.all(out == -1.5)


def test_tone_peaks_in_its_band():
    sr = 16000
    t = np.arange(sr) / sr
    for f in (300.0, 1000.0, 3000.0):
        out = omel.log_mel(np.sin(2 * math.pi * f * t))
        band = int(np.argmax(out[:, 50]))
        fb = omel.filterbank()
        bin_f = int(round(f / (sr / 1024)))
        assert fb[bin_f, band] > 0, (f, band)


def test_filterbank_structure():
    fb = omel.filterbank()
    assert fb.shape == (513, 128)
    nnz = int((fb > 0).sum())
    assert 990 <= nnz <= 1020, nnz  # SURVEY: ~1006 nonzeros
    assert int((fb > 0).sum(1).max()) <= 2  # at most two filters overlap any bin
    # every band's support is contiguous and narrower than the kernel's 32-bin window
    for m in range(128):
        nz = np.nonzero(fb[:, m] > 0)[0]
        assert nz.size > 0 and nz[-1] - nz[0] + 1 == nz.size and nz.size <= 32


def test_host_filterbank_matches_oracle():
    from asrx import mel as amel

    fb32 = amel.mel_filterbank().numpy().astype(np.float64)
    fb64 = omel.filterbank()
    assert np.max(np.abs(fb32 - fb64)) < 5e-5  # float32 f_pts vs float64
    starts, w = amel.sparse_filterbank(amel.mel_filterbank())
    dense = np.zeros((513, 128))
    for m in range(128):
        s = int(starts[m])
        for i in range(32):
            if s + i < 513:
                dense[s + i, m] = float(w[m, i])
    assert np.allclose(dense, fb32)


def test_waveform_pool_exact_means():
    x = np.random.default_rng(0).standard_normal(480000)
    w = omel.waveform_feature(x)
    assert w.shape == (1, 3000)
    assert np.allclose(w[0], x.reshape(3000, 160).mean(1))


def test_stft_matches_torch():
    # torch.stft is available (torchaudio is not): pin the framing/window/centering restatement.
    x = np.random.default_rng(1).standard_normal(4000)
    ours = omel.power_spectrogram(x)
    st = torch.stft(torch.from_numpy(x), 1024, hop_length=160, window=torch.hann_window(1024, dtype=torch.float64),
                    center=True, pad_mode="constant", return_complex=True)
    ref = (st.abs() ** 2).numpy()
    assert ours.shape == ref.shape
    assert np.allclose(ours, ref, rtol=1e-9, atol=1e-9)
