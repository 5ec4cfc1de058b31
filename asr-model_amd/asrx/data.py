"""Real-data feature path: audio files -> device waveforms -> features.

Reference: load_wave (essentials.py:301-319) reads each file with soundfile.read(dtype='float32') and
peak-normalises it on the CPU; prepare_datasets.__getitem__ (998-1026) runs extract_features per clip
inside the Dataset, which moves each feature to cuda:0 on its own (essentials.py:491).

Here:
  * FLAC (LibriSpeech's format) is decoded by the native RFC 9639 decoder in libasrx
    (csrc/flac.cpp, every frame CRC-checked); WAV by features.read_wav;
  * read_audio(path) returns exactly what soundfile.read(path, dtype='float32') returns (int PCM scaled
    by 2^-(bits-1), 1-D for mono), so load_wave keeps the reference's per-clip semantics;
  * load_batch(paths) is the batched device path: the files of a batch are decoded on a thread pool
    (the C decoder runs outside the GIL), packed into one pinned int32 buffer, copied to the GPU in one
    non-blocking H2D transfer, and scaled + peak-normalised there by one kernel
    (asrx_pcm_normalize) -- the reference's per-sample CPU normalisation and .to(device) disappear;
  * prepare_datasets mirrors the reference Dataset (CSV metadata with `audio` / `sentence` columns).
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import os

import numpy as np
import torch

from . import lib

FLAC_MAGIC = b"fLaC"


def decode_flac(data: bytes):
    """In-memory FLAC -> (pcm int32 (channels, frames), rate, bits, md5 bytes) via asrx_flac_decode."""
    L = lib.load()
    buf = ctypes.create_string_buffer(data, len(data))
    frames, ch, rate, bits = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    md5 = ctypes.create_string_buffer(16)
    lib.check(L.asrx_flac_info(buf, len(data), ctypes.byref(frames), ctypes.byref(ch), ctypes.byref(rate),
                               ctypes.byref(bits), md5), "asrx_flac_info")
    out = np.empty((ch.value, frames.value), dtype=np.int32)
    lib.check(L.asrx_flac_decode(buf, len(data), out.ctypes.data, frames.value), "asrx_flac_decode")
    return out, rate.value, bits.value, md5.raw


def _read_pcm(path):
    """(pcm int32 (C, N), rate, bits) for FLAC, or (float32 (C, N), rate, 0) for WAV."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] == FLAC_MAGIC:
        pcm, rate, bits, _ = decode_flac(data)
        return pcm, rate, bits
    from .features import read_wav

    x, rate = read_wav(path)
    x = x.reshape(len(x), -1).T
    return np.ascontiguousarray(x), rate, 0


def read_audio(path):
    """soundfile.read(path, dtype='float32') for FLAC and WAV: (float32 (frames,) or (frames, C), rate)."""
    pcm, rate, bits = _read_pcm(path)
    if bits:
        x = (pcm.astype(np.float64) * (1.0 / float(1 << (bits - 1)))).astype(np.float32)
    else:
        x = pcm
    x = x.T
    return (np.ascontiguousarray(x[:, 0]) if x.shape[1] == 1 else np.ascontiguousarray(x)), rate


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        _POOL = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 8))
    return _POOL


def load_batch(paths, device="cuda", normalize=True, pad_to=None):
    """Decode a batch of audio files and bring them to the GPU as load_wave's waveforms.

    Returns (wave (B, C, N) float32 on `device`, zero past each clip, lengths (B,) int64, rates).  Each
    clip is scaled like soundfile float32 and (normalize=True) peak-normalised like load_wave's file
    branch (essentials.py:303-312), on the device."""
    decoded = list(_pool().map(_read_pcm, paths))
    B = len(decoded)
    C = max(p.shape[0] for p, _, _ in decoded)
    if any(p.shape[0] != C for p, _, _ in decoded):
        raise ValueError("load_batch: clips with different channel counts")
    N = max(p.shape[1] for p, _, _ in decoded)
    ld = max(N, pad_to or 0)
    is_float = any(bits == 0 for _, _, bits in decoded)  # WAV (already float32): stage float32
    host = torch.empty((B, C, N), dtype=torch.float32 if is_float else torch.int32,
                       pin_memory=torch.cuda.is_available())
    hn = host.numpy()
    scale = np.empty(B, dtype=np.float32)
    lengths = np.empty(B, dtype=np.int64)
    for b, (p, rate, bits) in enumerate(decoded):
        n = p.shape[1]
        lengths[b] = n
        if is_float and bits:  # integer PCM into a float batch: soundfile's float32 values
            hn[b, :, :n] = (p.astype(np.float64) * (1.0 / float(1 << (bits - 1)))).astype(np.float32)
            scale[b] = 1.0
        else:
            hn[b, :, :n] = p
            scale[b] = 1.0 / float(1 << (bits - 1)) if bits else 1.0
        hn[b, :, n:] = 0
    dev = torch.device(device)
    pcm = host.to(dev, non_blocking=True)
    sc = torch.from_numpy(scale).to(dev, non_blocking=True)
    ln = torch.from_numpy(lengths).to(dev, non_blocking=True)
    out = torch.empty((B, C, ld), dtype=torch.float32, device=dev)
    lib.require_gpu(pcm, out)
    lib.call("asrx_pcm_normalize", lib.ptr(pcm), int(is_float), B, C, N, lib.ptr(ln), lib.ptr(sc), lib.ptr(out),
             ld, int(normalize), lib.stream())
    return out, torch.from_numpy(lengths), [r for _, r, _ in decoded]


class prepare_datasets(torch.utils.data.Dataset):  # noqa: N801  (reference class name)
    """essentials.prepare_datasets (essentials.py:998-1026): a CSV with `audio` (path relative to
    data_dir) and `sentence` columns; __getitem__ -> extract_features(batch, tokenizer, **extract_args)."""

    def __init__(self, metadata_file, data_dir, tokenizer=None, extract_args=None):
        import pandas as pd

        self.metadata = pd.read_csv(metadata_file)
        self.data_dir = data_dir
        self.tokenizer = tokenizer
        self.extract_args = extract_args if extract_args is not None else {}

    def __len__(self):
        return len(self.metadata)

    def __getitem__(self, idx):
        from .features import extract_features

        if torch.is_tensor(idx):
            idx = idx.tolist()
        row = self.metadata.iloc[idx]
        batch_input = {"audio": os.path.join(self.data_dir, row["audio"]), "transcription": row["sentence"]}
        return extract_features(batch_input, tokenizer=self.tokenizer, **self.extract_args)


def extract_features_batch(batches, tokenizer=None, spectrogram=False, waveform=False, pitch=False, phase=False,
                           hop_length=160, sample_rate=16000, mels=128, **unsupported):
    """extract_features (essentials.py:423-521) over a list of {"audio": path, "transcription"|"sentence"}
    dicts, with the audio of all of them loaded by one load_batch (one H2D copy, device normalisation).
    Returns the same per-clip feature dicts as extract_features (for DataCollator)."""
    from . import mel as _mel

    if any(unsupported.get(k) for k in ("harmonics", "aperiodics", "pitch_tokens")):
        raise NotImplementedError("harmonics / aperiodics / pitch_tokens: see extract_features")
    if hop_length != _mel.HOP or sample_rate != _mel.SAMPLE_RATE or mels != _mel.N_MELS:
        raise NotImplementedError("the HIP front end is built for hop 160, 16 kHz, 128 mels")
    wave, lengths, _ = load_batch([b["audio"] for b in batches])
    pitch_of, phase_of = {}, {}
    if pitch or phase:  # one batched GPU dio (+ stonemask) per group of equal-length clips
        from .pitch import dio, stonemask

        groups = {}
        for i in range(len(batches)):
            groups.setdefault(int(lengths[i]), []).append(i)
        for n, idx in groups.items():
            x = wave[idx, 0, :n].contiguous()
            if pitch:  # dio(x, fs, frame_period) binds frame_period to f0_floor (asrx/pitch.py)
                fp = hop_length / sample_rate * 1000
                f0, t = dio(x, sample_rate, fp)
                f0 = stonemask(x, f0, t, sample_rate)
                for j, i in enumerate(idx):
                    pitch_of[i] = f0[j].to(torch.float32).unsqueeze(0)
            if phase:
                f0, t = dio(x, sample_rate, frame_period=hop_length / sample_rate * 1000)
                tframe = torch.mean(t[1:] - t[:-1])
                ph = torch.remainder(torch.cumsum(2 * torch.pi * f0 * tframe, dim=-1), 2 * torch.pi)
                for j, i in enumerate(idx):
                    phase_of[i] = ph[j].to(torch.float32)
    out = []
    for i, b in enumerate(batches):
        n = int(lengths[i])
        audio = wave[i, 0, :n].contiguous()
        labels = tokenizer.encode(b["transcription" if "transcription" in b else "sentence"]) if tokenizer else []
        s_tensor = w_tensor = None
        if spectrogram:
            s_tensor = _mel.logmel(audio.unsqueeze(0), layout="BMF")[0]
        if waveform:
            target = int((n / sample_rate) * (sample_rate // hop_length))
            if n > target and n == target * hop_length:
                _, w_tensor = _mel.logmel(audio.unsqueeze(0), layout="BMF", pool=True)
            elif n > target and target > 0:  # as features.extract_features: wave_pool needs 0 < target < n
                w_tensor = _mel.wave_pool(audio.unsqueeze(0), target)
            else:
                w_tensor = torch.nn.functional.interpolate(audio.view(1, 1, -1), size=target, mode="linear",
                                                           align_corners=False)[0]
        out.append({"waveform": w_tensor, "spectrogram": s_tensor, "pitch_tokens": None, "pitch": pitch_of.get(i),
                    "harmonic": None, "aperiodic": None, "labels": labels, "phase": phase_of.get(i)})
    return out
