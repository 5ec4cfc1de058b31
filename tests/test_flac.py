"""Native FLAC decoder (csrc/flac.cpp, RFC 9639) behind load_wave's file branch (essentials.py:301-319)
and prepare_datasets (998-1026).  No FLAC files, libFLAC or soundfile exist in this image: streams are
made by the test-only encoder tests/flac_encode.py, exercising every format feature the decoder
handles, and checked three ways: decoded PCM == the encoder's input, the MD5 of the decoded samples
(hashlib, FLAC's interleaved little-endian convention) == STREAMINFO's MD5, and corrupted frames are
rejected by the CRC checks.  Host code only: runs without a GPU."""
import hashlib
import os

import numpy as np
import pytest

import flac_encode as fe


def _decode(data):
    from asrx.data import decode_flac

    return decode_flac(data)


def _md5(pcm, bps):
    nb = (bps + 7) // 8
    return hashlib.md5(b"".join(int(v).to_bytes(nb, "little", signed=True) for v in pcm.T.reshape(-1))).digest()


def _signal(ch, n, bps, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) - 1
    x = np.stack([0.6 * np.sin(2 * np.pi * (0.01 + 0.003 * c) * t) + 0.05 * rng.standard_normal(n)
                  for c in range(ch)])
    return np.clip(np.round(x * amp), -amp - 1, amp).astype(np.int64)


def _check(data, pcm, bps):
    out, rate, bits, md5 = _decode(data)
    assert bits == bps and out.shape == pcm.shape
    assert np.array_equal(out.astype(np.int64), pcm)
    assert md5 == _md5(out.astype(np.int64), bps)
    return rate


KINDS = [("verbatim", {}), ("fixed", {"order": 0}), ("fixed", {"order": 1}), ("fixed", {"order": 2}),
         ("fixed", {"order": 3}), ("fixed", {"order": 4}), ("lpc", {"order": 1}), ("lpc", {"order": 8}),
         ("lpc", {"order": 32, "prec": 15}), ("fixed", {"order": 2, "method": 1}),
         ("fixed", {"order": 2, "porder": 0}), ("fixed", {"order": 2, "escape": 1}),
         ("lpc", {"order": 4, "method": 1, "escape": 0, "porder": 3})]


@pytest.mark.parametrize("kind,kw", KINDS)
def test_subframe_types_mono16(kind, kw):
    pcm = _signal(1, 5000, 16, 1)
    data = fe.encode(pcm, 16000, 16, block=1152, plan=lambda f, c: (kind, kw))
    assert _check(data, pcm, 16) == 16000


@pytest.mark.parametrize("mode", [1, 8, 9, 10])
@pytest.mark.parametrize("bps", [8, 12, 16, 20, 24])
def test_stereo_modes_and_depths(mode, bps):
    pcm = _signal(2, 3000, bps, bps + mode)
    data = fe.encode(pcm, 44100, bps, block=576, stereo=lambda f: mode,
                     plan=lambda f, c: [("fixed", {"order": 2}), ("lpc", {"order": 6})][f % 2])
    _check(data, pcm, bps)


def test_constant_wasted_bits_and_odd_codes():
    """CONSTANT subframes (silence), wasted low bits, block-size codes 6/7 (the short last frame),
    frame numbers past 127 (multi-byte UTF-8), sample rate / size taken from STREAMINFO (codes 0)."""
    n = 192 * 140 + 77
    pcm = _signal(1, n, 16, 3)
    pcm[0, :192 * 3] = 0                     # constant frames
    pcm[0, 192 * 10:192 * 20] &= ~0x7        # 3 wasted bits in frames 10..19
    plan = lambda f, c: (("constant", {}) if f < 3 else  # noqa: E731
                         ("fixed", {"order": 1, "wasted": 3}) if 10 <= f < 20 else ("fixed", {"order": 2}))
    data = fe.encode(pcm, 12345, 16, block=192, plan=plan, force_codes0=True)
    assert _check(data, pcm, 16) == 12345


@pytest.mark.parametrize("rate", [8000, 16000, 22050, 44100, 96000, 7000, 11025, 50000])
def test_rate_codes_and_variable_blocking(rate):
    pcm = _signal(1, 9000, 16, rate)
    data = fe.encode(pcm, rate, 16, block=1024, variable=True, plan=lambda f, c: ("lpc", {"order": 4 + f % 5}))
    assert _check(data, pcm, 16) == rate


def test_corruption_is_detected():
    pcm = _signal(1, 4000, 16, 9)
    data = bytearray(fe.encode(pcm, 16000, 16, block=1024))
    _check(bytes(data), pcm, 16)
    bad = bytearray(data)
    bad[len(bad) // 2] ^= 0x10  # inside a frame body -> CRC-16 mismatch
    with pytest.raises(RuntimeError, match="CRC|truncated|reserved|sync|invalid"):
        _decode(bytes(bad))
    with pytest.raises(RuntimeError, match="fLaC"):
        _decode(b"RIFF" + bytes(60))
    with pytest.raises(RuntimeError):
        _decode(bytes(data[:len(data) - 5]))


def test_load_wave_flac_matches_soundfile_semantics(tmp_path):
    """load_wave(path) on FLAC: soundfile float32 values (pcm / 2^(bits-1)), then the reference's peak
    normalisation (mono by max|x|; multi-channel by the per-channel max of x)."""
    from asrx.features import load_wave

    mono = _signal(1, 4000, 16, 21)
    p1 = tmp_path / "m.flac"
    p1.write_bytes(fe.encode(mono, 16000, 16, block=4096))
    w, sr = load_wave(str(p1))
    x = (mono[0] / 32768.0).astype(np.float32)
    assert sr == 16000 and w.dtype == torch_float32()
    assert np.array_equal(w.numpy(), x / np.float32(np.abs(x).max()))
    st = _signal(2, 3000, 24, 22)
    p2 = tmp_path / "s.flac"
    p2.write_bytes(fe.encode(st, 16000, 24, block=1152, stereo=lambda f: 10))
    w2, _ = load_wave(str(p2))
    x2 = (st.T / float(1 << 23)).astype(np.float32)
    assert np.array_equal(w2.numpy(), (x2 / x2.max(axis=0)).T)


def torch_float32():
    import torch

    return torch.float32


def test_prepare_datasets_reads_flac_rows(tmp_path, monkeypatch):
    """prepare_datasets (essentials.py:998-1026): CSV rows -> extract_features(audio path, sentence);
    the feature extraction itself needs the GPU, so it is stubbed to capture the call."""
    import pandas as pd

    from asrx import data, features

    pcm = _signal(1, 1600, 16, 5)
    (tmp_path / "a.flac").write_bytes(fe.encode(pcm, 16000, 16))
    pd.DataFrame({"audio": ["a.flac"], "sentence": ["hello world"]}).to_csv(tmp_path / "meta.csv", index=False)
    seen = {}

    def fake(batch, tokenizer=None, **kw):
        seen.update(batch=batch, kw=kw, wave=features.load_wave(batch["audio"])[0])
        return {"ok": True}

    monkeypatch.setattr(features, "extract_features", fake)
    ds = data.prepare_datasets(str(tmp_path / "meta.csv"), str(tmp_path), tokenizer=None,
                               extract_args={"spectrogram": True})
    assert len(ds) == 1 and ds[0] == {"ok": True}
    assert seen["batch"]["transcription"] == "hello world" and seen["kw"] == {"spectrogram": True}
    assert os.path.basename(seen["batch"]["audio"]) == "a.flac" and seen["wave"].shape == (1600,)


def test_streaminfo_total_is_bounded_by_stream_size():
    """A STREAMINFO claiming ~2^36 samples (hostile or corrupt) is refused before the caller allocates
    channels x total samples (the decode would only fail after that allocation)."""
    pcm = _signal(1, 4000, 16, 5)
    data = bytearray(fe.encode(pcm, 16000, 16, block=1024))
    si = 8  # "fLaC" + 4-byte metadata block header
    word = int.from_bytes(data[si + 10:si + 18], "big")  # rate 20 | channels-1 3 | bps-1 5 | total 36
    word |= (1 << 36) - 1
    data[si + 10:si + 18] = word.to_bytes(8, "big")
    with pytest.raises(RuntimeError, match="claims"):
        _decode(bytes(data))
