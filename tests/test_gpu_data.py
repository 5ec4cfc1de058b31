"""Batched device audio path (asrx.data.load_batch): FLAC clips decoded on a
thread pool, one pinned H2D copy, scaling + peak normalisation on the GPU (asrx_pcm_normalize) --
bit-identical to load_wave's per-clip CPU semantics (essentials.py:301-319), zero past each clip;
and extract_features_batch giving the same features as per-clip extract_features."""
import numpy as np
import pytest
import torch

import flac_encode as fe

pytestmark = pytest.mark.gpu


def _clip(n, seed, bps=16, ch=1):
    rng = np.random.default_rng(seed)
    amp = (1 << (bps - 1)) - 1
    x = 0.5 * np.sin(2 * np.pi * 0.013 * np.arange(n)) * (0.5 + rng.random()) + 0.05 * rng.standard_normal((ch, n))
    return np.clip(np.round(x * amp), -amp - 1, amp).astype(np.int64)


def test_load_batch_matches_load_wave(cuda, tmp_path):
    from asrx.data import load_batch
    from asrx.features import load_wave

    paths = []
    for i, n in enumerate([16000, 12345, 20001, 800]):
        p = tmp_path / f"c{i}.flac"
        p.write_bytes(fe.encode(_clip(n, i), 16000, 16, block=4096))
        paths.append(str(p))
    z = tmp_path / "silence.flac"  # all-zero clip: no normalisation (max 0)
    z.write_bytes(fe.encode(np.zeros((1, 500), dtype=np.int64), 16000, 16))
    paths.append(str(z))
    wave, lengths, rates = load_batch(paths, device=cuda)
    torch.cuda.synchronize()
    w = wave.cpu()
    assert w.shape == (5, 1, 20001) and rates == [16000] * 5
    for i, p in enumerate(paths):
        ref, _ = load_wave(p)
        n = ref.shape[-1]
        assert int(lengths[i]) == n
        assert torch.equal(w[i, 0, :n], ref)
        assert bool((w[i, 0, n:] == 0).all())


def test_load_batch_stereo_quirk(cuda, tmp_path):
    from asrx.data import load_batch
    from asrx.features import load_wave

    paths = []
    for i in range(2):
        p = tmp_path / f"s{i}.flac"
        p.write_bytes(fe.encode(_clip(3000 + 7 * i, 10 + i, bps=24, ch=2), 16000, 24, stereo=lambda f: 10))
        paths.append(str(p))
    wave, lengths, _ = load_batch(paths, device=cuda)
    for i, p in enumerate(paths):
        ref, _ = load_wave(p)  # per-channel max of x (not |x|), essentials.py:305-307
        assert torch.equal(wave[i, :, :ref.shape[-1]].cpu(), ref)


def test_extract_features_batch_matches_per_clip(cuda, tmp_path):
    from asrx import data, features

    class Tok:
        def encode(self, s):
            return [len(w) + 3 for w in s.split()]

    items = []
    for i, n in enumerate([48000, 32000]):
        p = tmp_path / f"f{i}.flac"
        p.write_bytes(fe.encode(_clip(n, 30 + i), 16000, 16))
        items.append({"audio": str(p), "transcription": f"clip number {i}"})
    batched = data.extract_features_batch(items, tokenizer=Tok(), spectrogram=True, waveform=True)
    for it, fb in zip(items, batched):
        f1 = features.extract_features(it, tokenizer=Tok(), spectrogram=True, waveform=True)
        assert fb["labels"] == f1["labels"]
        assert torch.equal(fb["spectrogram"], f1["spectrogram"])
        assert torch.equal(fb["waveform"], f1["waveform"])
