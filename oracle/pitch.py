"""float64 numpy restatement of the reference's pitch feature.

essentials.py:451-455 (extract_features, pitch=True):
    frame_period = hop_length / sample_rate * 1000
    f0, t = pw.dio(audio.numpy().astype(np.float64), sample_rate, frame_period)
    f0 = pw.stonemask(audio.numpy().astype(np.float64), f0, t, sample_rate)
pyworld's signature is dio(x, fs, f0_floor=71.0, f0_ceil=800.0, channels_in_octave=2.0,
frame_period=5.0, speed=1, allowed_range=0.1), so the third POSITIONAL argument is f0_floor: the
reference extracts pitch with f0_floor = 10.0 (hop 160 at 16 kHz) and the default 5 ms frame period
(1 + 1000 N / fs / 5 frames: 6001 for a 30 s clip).  Restated as called (reference_pitch), quirk
included; the phase branch (essentials.py:458-467) passes frame_period by keyword.

pyworld wraps the WORLD vocoder (C++, dio.cpp / stonemask.cpp / matlabfunctions.cpp).  Neither is
in /root/reference or importable here and the reference pins no version (no requirements file).
This file restates WORLD's published DIO (Morise et al., "Fast and reliable F0 estimation method
based on the period extraction of vocal fold vibration of singing voice and speech", AES 2009) and
StoneMask (instantaneous-frequency refinement) as released in WORLD 0.2.x-0.3.x, from the algorithm
description: the DC-removed signal is high-passed at 50 Hz (zero-phase raised-cosine low-cut design)
and, per candidate band (boundary f0 = f0_floor 2^((i+1)/channels_in_octave)), low-passed with a
Nuttall window of 4 round(fs / f0_b / 2) taps (delay compensated); the negative- and positive-going
zero crossings, peaks and dips of each band give four interval series, linearly interpolated to the
frame times (MATLAB interp1 with end-segment extrapolation); their mean is the band's candidate and
their standard deviation its score; out-of-band candidates are dropped; the best-scoring band wins per
frame; FixF0Contour (jump removal against allowed_range, removal of voiced runs shorter than the
minimum voice range, forward / backward extension of voiced sections through the candidates).
StoneMask: per frame, a Blackman window of 3 periods and its central difference, the spectrum and
the instantaneous frequency at the first min(fs/2/f0, 6) harmonics, amplitude-weighted mean; kept
only within 20 % of the input f0.  **Parity unpinned**: no pyworld / WORLD output exists here to check
against; the restatement is pinned by known-answer tests (tests/test_pitch.py: harmonic signals of
known f0, silence, the frame count) and the GPU path (asrx/pitch.py) is checked against it.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
from __future__ import annotations

import math

import numpy as np

K_CUTOFF = 50.0
K_MAX_VALUE = 100000.0
K_SAFE = 1e-12
K_FLOOR_STONEMASK = 40.0


def matlab_round(x):
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def suitable_fft_size(n):
    return int(2 ** (int(math.log(n) / math.log(2.0)) + 1))


def samples_for_dio(fs, x_length, frame_period):
    return int(1000.0 * x_length / fs / frame_period) + 1


def low_cut_filter(N, fft_size):
    """Zero-phase high-pass (delta minus a normalised raised-cosine low-pass of N taps), circular."""
    w = 0.5 - 0.5 * np.cos(np.arange(1, N + 1) * 2.0 * math.pi / (N + 1))
    w = -w / w.sum()
    c = (N - 1) // 2
    h = np.zeros(fft_size)
    h[:c + 1] = w[c:]          # taps 0 .. c
    h[fft_size - c:] = w[:c]   # taps -c .. -1
    h[0] += 1.0
    return h


def nuttall(n):
    t = np.arange(n) / (n - 1.0)
    return (0.355768 - 0.487396 * np.cos(2 * math.pi * t) + 0.144232 * np.cos(4 * math.pi * t)
            - 0.012604 * np.cos(6 * math.pi * t))


def spectrum_for_estimation(x, y_length, fs, fft_size):
    y = np.zeros(fft_size)
    y[:len(x)] = x
    y[:y_length] -= y[:y_length].mean()
    Y = np.fft.rfft(y)
    N = matlab_round(fs / K_CUTOFF) * 2 + 1
    return Y * np.fft.rfft(low_cut_filter(N, fft_size))


def filtered_signal(half, fft_size, Y, y_length):
    lp = np.zeros(fft_size)
    lp[:4 * half] = nuttall(4 * half)
    f = np.fft.irfft(Y * np.fft.rfft(lp), fft_size)
    return f[2 * half:2 * half + y_length]


def zero_crossings(sig, fs):
    """WORLD ZeroCrossingEngine: negative-going crossings of sig, linearly interpolated."""
    s = np.asarray(sig)
    idx = np.nonzero((s[:-1] > 0.0) & (s[1:] <= 0.0))[0] + 1
    if len(idx) < 2:
        return np.zeros(0), np.zeros(0)
    fine = idx - s[idx - 1] / (s[idx] - s[idx - 1])
    return (fine[:-1] + fine[1:]) / 2.0 / fs, fs / (fine[1:] - fine[:-1])


def interp1(x, y, xi):
    """MATLAB interp1 (linear) as WORLD's matlabfunctions: histc bins, end segments extrapolate."""
    n = len(x)
    k = np.searchsorted(x, xi, side="right")  # x[k-1] <= xi < x[k]
    k = np.clip(k, 1, n - 1)
    h = x[k] - x[k - 1]
    s = (xi - x[k - 1]) / h
    return y[k - 1] + s * (y[k] - y[k - 1])


def band_candidates(boundary_f0, fs, Y, y_length, fft_size, f0_floor, f0_ceil, times):
    f = filtered_signal(matlab_round(fs / boundary_f0 / 2.0), fft_size, Y, y_length)
    events = [zero_crossings(f, fs)]
    f = -f
    events.append(zero_crossings(f, fs))
    d = f[:-1] - f[1:]
    events.append(zero_crossings(d, fs))
    events.append(zero_crossings(-d, fs))
    nfr = len(times)
    if any(len(loc) < 3 for loc, _ in events):  # CheckEvent(number_of_intervals - 2) on each series
        return np.zeros(nfr), np.full(nfr, K_MAX_VALUE)
    sets = np.stack([interp1(loc, iv, times) for loc, iv in events])
    cand = sets.mean(0)
    score = np.sqrt(((sets - cand) ** 2).sum(0) / 3.0)
    bad = (cand > boundary_f0) | (cand < boundary_f0 / 2.0) | (cand > f0_ceil) | (cand < f0_floor)
    cand[bad] = 0.0
    score[bad] = K_MAX_VALUE
    return cand, score


def select_best(ref, cands, allowed_range):
    best, err = 0.0, allowed_range
    for c in cands:
        e = abs(ref - c) / ref
        if e > err:
            continue
        best, err = c, e
    return best


def fix_f0_contour(frame_period, cands, best, f0_floor, allowed_range):
    n = len(best)
    vmin = int(0.5 + 1000.0 / frame_period / f0_floor) * 2 + 1
    if n <= vmin:
        return best.copy()
    # step 1: edges zeroed, jumps removed
    base = best.copy()
    base[:vmin] = 0.0
    base[n - vmin:] = 0.0
    s1 = np.zeros(n)
    for i in range(vmin, n):
        s1[i] = base[i] if abs((base[i] - base[i - 1]) / (K_SAFE + base[i])) < allowed_range else 0.0
    # step 2: voiced runs shorter than the minimum voice range removed
    s2 = s1.copy()
    c = (vmin - 1) // 2
    for i in range(c, n - c):
        if (s1[i - c:i + c + 1] == 0.0).any():
            s2[i] = 0.0
    # voiced section boundaries
    pos, neg = [], []
    for i in range(1, n):
        if s2[i] == 0.0 and s2[i - 1] != 0.0:
            neg.append(i - 1)
        elif s2[i - 1] == 0.0 and s2[i] != 0.0:
            pos.append(i)
    # step 3: extend each voiced section forwards through the candidates
    s3 = s2.copy()
    for i, start in enumerate(neg):
        limit = n - 1 if i == len(neg) - 1 else neg[i + 1]
        for j in range(start, limit):
            s3[j + 1] = select_best(s3[j], cands[:, j + 1], allowed_range)
            if s3[j + 1] == 0.0:
                break
    # step 4: and backwards
    s4 = s3.copy()
    for i in range(len(pos) - 1, -1, -1):
        limit = 1 if i == 0 else pos[i - 1]
        for j in range(pos[i], limit, -1):
            s4[j - 1] = select_best(s4[j], cands[:, j - 1], allowed_range)
            if s4[j - 1] == 0.0:
                break
    return s4


def dio(x, fs, f0_floor=71.0, f0_ceil=800.0, channels_in_octave=2.0, frame_period=5.0, speed=1,
        allowed_range=0.1):
    """pyworld.dio (speed 1: no decimation).  Returns (f0, temporal_positions)."""
    if speed != 1:
        raise NotImplementedError("dio: speed != 1 (decimation) is not restated")
    x = np.asarray(x, dtype=np.float64)
    n_bands = 1 + int(math.log(f0_ceil / f0_floor) / math.log(2.0) * channels_in_octave)
    bf0 = [f0_floor * 2.0 ** ((i + 1) / channels_in_octave) for i in range(n_bands)]
    y_length = 1 + len(x)
    fft_size = suitable_fft_size(y_length + matlab_round(fs / K_CUTOFF) * 2 + 1
                                 + 4 * int(1.0 + fs / bf0[0] / 2.0))
    nfr = samples_for_dio(fs, len(x), frame_period)
    times = np.arange(nfr) * frame_period / 1000.0
    Y = spectrum_for_estimation(x, y_length, fs, fft_size)
    cands = np.zeros((n_bands, nfr))
    scores = np.zeros((n_bands, nfr))
    for i, b in enumerate(bf0):
        cands[i], scores[i] = band_candidates(b, fs, Y, y_length, fft_size, f0_floor, f0_ceil, times)
    best_idx = np.zeros(nfr, dtype=np.int64)
    for j in range(nfr):  # first band with the smallest score (strict improvement)
        bi, bs = 0, scores[0, j]
        for i in range(1, n_bands):
            if bs > scores[i, j]:
                bi, bs = i, scores[i, j]
        best_idx[j] = bi
    best = cands[best_idx, np.arange(nfr)]
    return fix_f0_contour(frame_period, cands, best, f0_floor, allowed_range), times


def _refined_f0(x, fs, t, f0):
    if f0 <= K_FLOOR_STONEMASK or f0 > fs / 12.0:
        return 0.0
    half = int(1.5 * fs / f0 + 1.0)
    wl = 2 * half + 1
    wlt = (2.0 * half + 1.0) / fs
    bt = (np.arange(wl) - half) / fs
    fft_size = int(2.0 ** (2.0 + int(math.log(half * 2.0 + 1.0) / math.log(2.0))))
    idx = np.array([matlab_round((t + b) * fs) for b in bt])
    idx = np.clip(idx - 1, 0, len(x) - 1)
    mw = 0.42 + 0.5 * np.cos(2.0 * math.pi * bt / wlt) + 0.08 * np.cos(4.0 * math.pi * bt / wlt)
    dw = np.empty(wl)
    dw[0] = -mw[1] / 2.0
    dw[1:-1] = -(mw[2:] - mw[:-2]) / 2.0
    dw[-1] = mw[-2] / 2.0
    seg = x[idx]
    M = np.fft.rfft(seg * mw, fft_size)
    Dsp = np.fft.rfft(seg * dw, fft_size)
    power = M.real ** 2 + M.imag ** 2
    num = M.real * Dsp.imag - M.imag * Dsp.real
    nh = min(int(fs / 2.0 / f0), 6)
    amp_sum = if_sum = 0.0
    for i in range(nh):
        k = matlab_round(f0 * fft_size / fs * (i + 1))
        inst = 0.0 if power[k] == 0.0 else k * fs / fft_size + num[k] / power[k] * fs / 2.0 / math.pi
        a = math.sqrt(power[k])
        amp_sum += a * (i + 1)
        if_sum += a * inst
    mean_f0 = if_sum / (amp_sum + K_SAFE)
    return f0 if abs(mean_f0 - f0) > f0 * 0.2 else mean_f0


def stonemask(x, f0, temporal_positions, fs):
    x = np.asarray(x, dtype=np.float64)
    return np.array([_refined_f0(x, fs, t, f) for t, f in zip(temporal_positions, f0)])


def reference_pitch(audio, sample_rate=16000, hop_length=160):
    """essentials.py:451-455 as written: dio(x, fs, frame_period) -> f0_floor = frame_period."""
    frame_period = hop_length / sample_rate * 1000
    x = np.asarray(audio, dtype=np.float64)
    f0, t = dio(x, sample_rate, frame_period)
    return stonemask(x, f0, t, sample_rate)
