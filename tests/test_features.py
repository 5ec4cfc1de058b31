"""The reference-facing feature boundary: DataCollator semantics (CPU) and extract_features on the
HIP log-mel kernel (GPU), checked against the oracle."""
import numpy as np
import pytest
import torch


class _Tok:
    def encode(self, text):
        return [3 + (ord(c) % 50) for c in text]


def test_data_collator_padding():
    from asrx.features import DataCollator

    feats = [{"labels": [5, 6, 7], "spectrogram": torch.ones(128, 4), "waveform": torch.ones(1, 3)},
             {"labels": [9], "spectrogram": torch.full((128, 6), 2.0), "waveform": torch.ones(1, 5)}]
    b = DataCollator(tokenizer=None)(feats)
    assert b["text_ids"].tolist() == [[1, 5, 6, 7], [1, 9, 0, 0]]
    assert b["labels"].tolist() == [[5, 6, 7, 2], [9, 2, 0, 0]]
    assert b["spectrogram"].shape == (2, 128, 6)
    assert torch.all(b["spectrogram"][0, :, 4:] == 0) and torch.all(b["spectrogram"][1] == 2.0)
    assert b["waveform"].shape == (2, 1, 5)


def test_extract_features_out_of_scope_streams():
    from asrx.features import extract_features

    with pytest.raises(NotImplementedError):
        extract_features({"audio": {"array": np.zeros(160), "sampling_rate": 16000}, "sentence": "a"},
                         tokenizer=_Tok(), pitch=True)


@pytest.mark.gpu
def test_extract_features_matches_oracle(cuda):
    from asrx.features import extract_features
    from oracle import mel as omel

    rng = np.random.default_rng(3)
    audio = (rng.standard_normal(16000) * 0.1).astype(np.float32)
    out = extract_features({"audio": {"array": audio, "sampling_rate": 16000}, "transcription": "hello"},
                           tokenizer=_Tok(), spectrogram=True, waveform=True)
    assert out["labels"] == _Tok().encode("hello")
    s = out["spectrogram"].cpu().numpy()
    assert s.shape == (128, 101)
    assert np.abs(s - omel.log_mel(audio.astype(np.float64))).max() < 2e-4
    w = out["waveform"].cpu().numpy()
    assert w.shape == (1, 100)
    assert np.abs(w - omel.waveform_feature(audio.astype(np.float64))).max() < 1e-6
