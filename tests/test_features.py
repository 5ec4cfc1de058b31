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

    for kw in ("harmonics", "aperiodics", "pitch_tokens"):  # cheaptrick / d4c streams stay out of scope
        with pytest.raises(NotImplementedError):
            extract_features({"audio": {"array": np.zeros(160), "sampling_rate": 16000}, "sentence": "a"},
                             tokenizer=_Tok(), **{kw: True})


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


def _write_wav(path, frames, rate, tag, bits, raw):
    ch = frames.shape[1] if frames.ndim > 1 else 1
    fmt = (tag.to_bytes(2, "little") + ch.to_bytes(2, "little") + rate.to_bytes(4, "little")
           + (rate * ch * bits // 8).to_bytes(4, "little") + (ch * bits // 8).to_bytes(2, "little")
           + bits.to_bytes(2, "little"))
    body = b"WAVE" + b"fmt " + len(fmt).to_bytes(4, "little") + fmt + b"LIST" + (3).to_bytes(4, "little") + b"abc\0"
    body += b"data" + len(raw).to_bytes(4, "little") + raw
    with open(path, "wb") as f:
        f.write(b"RIFF" + len(body).to_bytes(4, "little") + body)


def test_load_wave_file_branch(tmp_path):
    """load_wave(path) (essentials.py:301-313): PCM16 / PCM24 / float32 WAV decoded as soundfile
    scales it, then peak-normalised (mono: max|x|; stereo: per-channel max of x, channels-first);
    an odd-sized chunk before `data` is skipped with its pad byte."""
    import wave

    from asrx.features import load_wave

    rng = np.random.default_rng(0)
    pcm = (rng.standard_normal(1000) * 3000).astype("<i2")
    p16 = str(tmp_path / "m16.wav")
    with wave.open(p16, "wb") as w:  # stdlib writer for the 16-bit case
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(pcm.tobytes())
    x, sr = load_wave(p16)
    ref = pcm.astype(np.float32) / 32768.0
    assert sr == 16000 and x.dtype == torch.float32 and x.shape == (1000,)
    np.testing.assert_allclose(x.numpy(), ref / np.abs(ref).max(), rtol=1e-6, atol=1e-7)

    v24 = rng.integers(-(1 << 23), 1 << 23, 600)
    raw24 = b"".join(int(v & 0xFFFFFF).to_bytes(3, "little") for v in v24)
    p24 = str(tmp_path / "m24.wav")
    _write_wav(p24, v24, 22050, 1, 24, raw24)
    x, sr = load_wave(p24)
    ref = v24 / float(1 << 23)
    assert sr == 22050
    np.testing.assert_allclose(x.numpy(), ref / np.abs(ref).max(), rtol=1e-6, atol=1e-7)

    st = (rng.standard_normal((500, 2)) * 0.3).astype("<f4")
    st[0] = [0.9, 0.7]
    pf = str(tmp_path / "stereo_f32.wav")
    _write_wav(pf, st, 8000, 3, 32, st.tobytes())
    x, sr = load_wave(pf)
    assert sr == 8000 and x.shape == (2, 500)
    np.testing.assert_allclose(x.numpy(), (st / st.max(axis=0)).T, rtol=1e-6)

    bad = str(tmp_path / "x.flac")
    open(bad, "wb").write(b"fLaC" + bytes(40))  # FLAC marker but no valid STREAMINFO (tests/test_flac.py)
    with pytest.raises(RuntimeError, match="asrx_flac"):
        load_wave(bad)
    other = str(tmp_path / "x.ogg")
    open(other, "wb").write(b"OggS" + bytes(40))
    with pytest.raises(NotImplementedError):
        load_wave(other)
    with pytest.raises(TypeError):
        load_wave(3)
