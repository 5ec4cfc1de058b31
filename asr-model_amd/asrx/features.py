"""Drop-in replacements for the reference's feature boundary (essentials.py:423-574):
`extract_features(batch, tokenizer, ...)` and `DataCollator(tokenizer)(features)`, same signatures,
keys and layouts.  The spectrogram and waveform features run on the HIP log-mel kernel; the
pyworld-based streams (pitch, harmonics, aperiodics, phase, pitch tokens) are out of scope
(CPU vocoder analysis, pyworld is not installed) and raise.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List

import torch

from . import mel as _mel

_DEVICE = torch.device("cuda:0")


def load_wave(audio, sample_rate=16000):
    """essentials.load_wave (essentials.py:301-319) for the in-memory dict branch.  The file-path
    branch needs soundfile, which is absent here: decode the file to a dict first."""
    if isinstance(audio, dict):
        return torch.as_tensor(audio["array"]).float(), audio["sampling_rate"]
    if isinstance(audio, str):
        raise NotImplementedError("load_wave(path): soundfile is not installed; pass {'array', 'sampling_rate'}")
    raise TypeError("Invalid wave_data format.")


def extract_features(batch, tokenizer=None, spectrogram=False, pitch=False, waveform=False, harmonics=False,
                     aperiodics=False, phase=False, hilbert=False, pitch_tokens=False, hop_length=160,
                     sample_rate=16000, mels=128):
    if pitch or harmonics or aperiodics or phase or pitch_tokens:
        raise NotImplementedError("pitch / harmonics / aperiodics / phase / pitch_tokens use pyworld "
                                  "(essentials.py:360-467): out of scope, pass a precomputed f0 track instead")
    if hop_length != _mel.HOP or sample_rate != _mel.SAMPLE_RATE or mels != _mel.N_MELS:
        raise NotImplementedError("the HIP front end is built for hop 160, 16 kHz, 128 mels (the reference's "
                                  "only configuration, model.py:733-744)")
    labels = tokenizer.encode(batch["transcription" if "transcription" in batch else "sentence"])
    audio, _ = load_wave(batch["audio"], sample_rate)
    audio = audio.to(_DEVICE, torch.float32).contiguous()
    s_tensor = w_tensor = None
    if spectrogram:
        s_tensor = _mel.logmel(audio.unsqueeze(0), layout="BMF")[0]  # (128, 1 + N // 160)
    if waveform:
        n = audio.shape[-1]
        target = int((n / sample_rate) * (sample_rate // hop_length))
        if n > target and n == target * hop_length:
            _, pooled = _mel.logmel(audio.unsqueeze(0), layout="BMF", pool=True)
            w_tensor = pooled  # (1, target)
        elif n > target:
            w_tensor = torch.nn.functional.adaptive_avg_pool1d(audio.view(1, 1, -1), target)[0]
        else:
            w_tensor = torch.nn.functional.interpolate(audio.view(1, 1, -1), size=target, mode="linear",
                                                       align_corners=False)[0]
    return {"waveform": w_tensor, "spectrogram": s_tensor, "pitch_tokens": None, "pitch": None, "harmonic": None,
            "aperiodic": None, "labels": labels, "phase": None}


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
