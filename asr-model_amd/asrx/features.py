"""Drop-in replacements for the reference's feature boundary (essentials.py:423-574):
`extract_features(batch, tokenizer, ...)` and `DataCollator(tokenizer)(features)`, same signatures,
keys and layouts.  The spectrogram and waveform features run on the HIP log-mel kernel; pitch (dio +
stonemask, essentials.py:451-455) and phase (dio, 458-467) on the GPU pitch kernels (asrx/pitch.py);
harmonics / aperiodics (cheaptrick / d4c) and pitch tokens stay out of scope and
raise.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List

import numpy as np
import torch

from . import mel as _mel

_DEVICE = torch.device("cuda:0")


def read_wav(path):
    """RIFF/WAVE decode to float32 (frames, channels) the way soundfile.read(path, dtype='float32')
    returns it: integer PCM scaled by 2^-(bits-1) (8-bit PCM is unsigned, offset 128), IEEE float
    passed through; WAVE_FORMAT_EXTENSIBLE resolved through its sub-format.  Returns (array, rate);
    the array is 1-D for mono, as soundfile returns it."""
    raw = open(path, "rb").read()
    if len(raw) < 12 or raw[:4] != b"RIFF" or raw[8:12] != b"WAVE":
        raise NotImplementedError(f"load_wave({path!r}): FLAC (asrx.data) and RIFF/WAVE files are decoded here "
                                  "(soundfile's other formats are not installed)")
    fmt = data = None
    pos = 12
    while pos + 8 <= len(raw):
        cid, size = raw[pos:pos + 4], int.from_bytes(raw[pos + 4:pos + 8], "little")
        body = raw[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError(f"{path!r}: WAVE file without fmt/data chunks")
    tag, ch, rate = int.from_bytes(fmt[0:2], "little"), int.from_bytes(fmt[2:4], "little"), int.from_bytes(fmt[4:8], "little")
    bits = int.from_bytes(fmt[14:16], "little")
    if tag == 0xFFFE and len(fmt) >= 26:
        tag = int.from_bytes(fmt[24:26], "little")
    width = bits // 8
    n = len(data) // (width * ch)
    buf = data[:n * width * ch]
    if tag == 3 and bits in (32, 64):
        x = np.frombuffer(buf, dtype="<f4" if bits == 32 else "<f8").astype(np.float32)
    elif tag == 1 and bits == 8:
        x = (np.frombuffer(buf, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == 1 and bits in (16, 32):
        x = np.frombuffer(buf, dtype="<i2" if bits == 16 else "<i4").astype(np.float64) / float(1 << (bits - 1))
        x = x.astype(np.float32)
    elif tag == 1 and bits == 24:
        b = np.frombuffer(buf, dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = (v.astype(np.float64) / float(1 << 23)).astype(np.float32)
    else:
        raise NotImplementedError(f"{path!r}: WAVE format tag {tag} with {bits}-bit samples is not supported")
    x = x.reshape(n, ch)
    return (x[:, 0].copy() if ch == 1 else x), rate


def load_wave(audio, sample_rate=16000):
    """essentials.load_wave (essentials.py:301-319).  File path: decoded like soundfile.read(path,
    dtype='float32') (FLAC by the native decoder of asrx.data, WAV by read_wav), then peak-normalised
    as the reference does -- mono by max|x|, multi-channel by the per-channel max of x (not of |x|,
    essentials.py:306) and returned channels-first.  Dict: the array as float32 with its own rate, not
    normalised.  asrx.data.load_batch is the batched device version of the file branch."""
    if isinstance(audio, str):
        from .data import read_audio

        wp, sample_rate = read_audio(audio)  # FLAC (native decoder) or WAV
        if wp.ndim > 1:
            abs_max = wp.max(axis=0)
            wp = wp / abs_max if any(abs_max > 0) else wp
            return torch.from_numpy(np.ascontiguousarray(wp.T)), sample_rate
        abs_max = float(np.abs(wp).max()) if wp.size else 0.0
        wp = wp / abs_max if abs_max > 0 else wp
        return torch.from_numpy(wp), sample_rate
    if isinstance(audio, dict):
        return torch.as_tensor(audio["array"]).float(), audio["sampling_rate"]
    raise TypeError("Invalid wave_data format.")


def extract_features(batch, tokenizer=None, spectrogram=False, pitch=False, waveform=False, harmonics=False,
                     aperiodics=False, phase=False, hilbert=False, pitch_tokens=False, hop_length=160,
                     sample_rate=16000, mels=128):
    if harmonics or aperiodics or pitch_tokens:
        raise NotImplementedError("harmonics / aperiodics / pitch_tokens use pyworld's cheaptrick / d4c "
                                  "(essentials.py:360-421): out of scope")
    if hop_length != _mel.HOP or sample_rate != _mel.SAMPLE_RATE or mels != _mel.N_MELS:
        raise NotImplementedError("the HIP front end is built for hop 160, 16 kHz, 128 mels (the reference's "
                                  "only configuration, model.py:733-744)")
    labels = tokenizer.encode(batch["transcription" if "transcription" in batch else "sentence"])
    audio, _ = load_wave(batch["audio"], sample_rate)
    audio = audio.to(_DEVICE, torch.float32).contiguous()
    s_tensor = w_tensor = p_tensor = ph_tensor = None
    if pitch:  # essentials.py:451-455, dio's third positional argument is f0_floor (asrx/pitch.py)
        from .pitch import reference_pitch

        p_tensor = reference_pitch(audio, sample_rate, hop_length).to(torch.float32).unsqueeze(0)
    if phase:  # essentials.py:458-467: dio at the hop's frame period, phase of the integrated f0
        from .pitch import dio

        f0, t = dio(audio, sample_rate, frame_period=hop_length / sample_rate * 1000)
        tframe = torch.mean(t[1:] - t[:-1])
        phi = torch.cumsum(2 * torch.pi * f0 * tframe, dim=0)
        ph_tensor = torch.remainder(phi, 2 * torch.pi).to(torch.float32)
    if spectrogram:
        s_tensor = _mel.logmel(audio.unsqueeze(0), layout="BMF")[0]  # (128, 1 + N // 160)
    if waveform:
        n = audio.shape[-1]
        target = int((n / sample_rate) * (sample_rate // hop_length))
        if n > target and n == target * hop_length:
            _, pooled = _mel.logmel(audio.unsqueeze(0), layout="BMF", pool=True)
            w_tensor = pooled  # (1, target)
        elif n > target and target > 0:
            w_tensor = _mel.wave_pool(audio.unsqueeze(0), target)  # (1, target), any clip length
        else:
            w_tensor = torch.nn.functional.interpolate(audio.view(1, 1, -1), size=target, mode="linear",
                                                       align_corners=False)[0]
    return {"waveform": w_tensor, "spectrogram": s_tensor, "pitch_tokens": None, "pitch": p_tensor, "harmonic": None,
            "aperiodic": None, "labels": labels, "phase": ph_tensor}


@dataclass
class DataCollator:
    """essentials.DataCollator (essentials.py:523-574): text_ids = [BOS] + y + PAD*, labels =
    y + [EOS] + PAD* (both max_len + 1 long); audio keys right-padded with 0 and stacked."""

    tokenizer: Any

    def __call__(self, features: List[Dict[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
        keys = set()
        for f in features:
            keys.update(f.keys())
        batch = {}
        pad, bos, eos = 0, 1, 2
        for key in keys:
            if key == "labels":
                lab = [f["labels"].tolist() if isinstance(f["labels"], torch.Tensor) else list(f["labels"])
                       for f in features]
                max_len = max(len(x) for x in lab)
                ids = [[bos] + x + [pad] * (max_len - len(x)) for x in lab]
                lbl = [x + [eos] + [pad] * (max_len - len(x)) for x in lab]
                batch["text_ids"] = torch.tensor(ids, dtype=torch.long)
                batch["labels"] = torch.tensor(lbl, dtype=torch.long)
            elif key in ("spectrogram", "waveform", "pitch", "pitch_tokens"):
                items = [f[key] for f in features if key in f and f[key] is not None]
                if not items:
                    continue
                items = [torch.as_tensor(t) for t in items]
                n = max(t.shape[-1] for t in items)
                batch[key] = torch.stack([torch.nn.functional.pad(t, (0, n - t.shape[-1]), value=pad)
                                          if t.shape[-1] < n else t for t in items])
        return batch
