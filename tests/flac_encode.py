"""Test-only FLAC encoder (RFC 9639), used to make FLAC fixtures for the native decoder
(asr-model_amd/csrc/flac.cpp): no FLAC files, libFLAC or soundfile exist in this image.

Every format feature the decoder handles can be forced per frame: CONSTANT / VERBATIM / FIXED (0-4) /
LPC subframes, wasted bits, Rice and Rice2 residuals with chosen partition orders and escape
partitions, the four stereo modes, fixed or variable blocking, block-size codes 1-15, sample-rate
codes 0-14, sample-size codes, multi-byte frame numbers.  STREAMINFO carries the MD5 of the PCM, which
the decoder test checks independently of this encoder (hashlib over the decoded samples).
"""
from __future__ import annotations

import hashlib

import numpy as np


class BitWriter:
    def __init__(self):
        self.buf = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, k):
        if k == 0:
            return
        v &= (1 << k) - 1
        self.acc = (self.acc << k) | v
        self.n += k
        while self.n >= 8:
            self.n -= 8
            self.buf.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def put_signed(self, v, k):
        self.put(v & ((1 << k) - 1), k)

    def unary(self, q):
        for _ in range(q):
            self.put(0, 1)
        self.put(1, 1)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def bytes(self):
        assert self.n == 0
        return bytes(self.buf)


def crc8(data):
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data):
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def utf8_num(v):
    if v < 0x80:
        return bytes([v])
    for nbytes, lead in ((2, 0xC0), (3, 0xE0), (4, 0xF0), (5, 0xF8), (6, 0xFC), (7, 0xFE)):
        bits = 5 * 1 + 6 * (nbytes - 1) if nbytes == 2 else (7 - nbytes) + 6 * (nbytes - 1)
        if nbytes == 7:
            bits = 36
        if v < (1 << bits):
            out = []
            for _ in range(nbytes - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            out.append(lead | v)
            return bytes(reversed(out))
    raise ValueError(v)


def zigzag(r):
    return 2 * r if r >= 0 else -2 * r - 1


def write_residual(bw, res, block, order, method=0, porder=None, escape_part=None):
    parts_max = 0
    while (block % (1 << (parts_max + 1)) == 0) and (block >> (parts_max + 1)) >= order and parts_max < 8:
        parts_max += 1
    porder = parts_max if porder is None else min(porder, parts_max)
    bw.put(method, 2)
    bw.put(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    i = 0
    for pt in range(1 << porder):
        cnt = (block >> porder) - (order if pt == 0 else 0)
        seg = [int(x) for x in res[i:i + cnt]]
        i += cnt
        if escape_part is not None and pt == escape_part:
            raw = max([abs(x).bit_length() + 1 for x in seg] + [1])
            bw.put(esc, pbits)
            bw.put(raw, 5)
            for x in seg:
                bw.put_signed(x, raw)
            continue
        u = np.array([zigzag(x) for x in seg], dtype=np.int64)
        costs = [int((u >> k).sum()) + len(seg) * (1 + k) for k in range(0, esc)]
        bk = int(np.argmin(costs))
        bw.put(bk, pbits)
        for x in seg:
            u = zigzag(x)
            bw.unary(u >> bk)
            bw.put(u & ((1 << bk) - 1), bk)


def fixed_residual(x, order):
    x = [int(v) for v in x]
    r = []
    for n in range(order, len(x)):
        p = {0: 0, 1: x[n - 1], 2: 2 * x[n - 1] - x[n - 2], 3: 3 * x[n - 1] - 3 * x[n - 2] + x[n - 3],
             4: 4 * x[n - 1] - 6 * x[n - 2] + 4 * x[n - 3] - x[n - 4]}[order]
        r.append(x[n] - p)
    return r


def write_subframe(bw, x, bps, kind, **kw):
    """x: int samples of this (possibly side) channel at bps bits."""
    x = [int(v) for v in x]
    wasted = kw.get("wasted", 0)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in x)
        x = [v >> wasted for v in x]
    sb = bps - wasted
    bw.put(0, 1)
    block = len(x)
    if kind == "constant":
        assert len(set(x)) == 1
        bw.put(0, 6)
    elif kind == "verbatim":
        bw.put(1, 6)
    elif kind == "fixed":
        bw.put(8 + kw["order"], 6)
    elif kind == "lpc":
        bw.put(32 + kw["order"] - 1, 6)
    if wasted:
        bw.put(1, 1)
        bw.unary(wasted - 1)
    else:
        bw.put(0, 1)
    if kind == "constant":
        bw.put_signed(x[0], sb)
    elif kind == "verbatim":
        for v in x:
            bw.put_signed(v, sb)
    elif kind == "fixed":
        o = kw["order"]
        for v in x[:o]:
            bw.put_signed(v, sb)
        write_residual(bw, fixed_residual(x, o), block, o, kw.get("method", 0), kw.get("porder"), kw.get("escape"))
    elif kind == "lpc":
        o, prec = kw["order"], kw.get("prec", 12)
        xs = np.array(x, dtype=np.float64)
        if block > 2 * o:
            A = np.stack([xs[o - 1 - j:block - 1 - j] for j in range(o)], 1)
            c, *_ = np.linalg.lstsq(A, xs[o:], rcond=None)
        else:
            c = np.zeros(o)
        cmax = max(np.abs(c).max(), 1e-9)
        shift = 0
        while shift < 15 and cmax * (1 << (shift + 1)) < (1 << (prec - 1)) - 1:
            shift += 1
        q = [int(np.clip(np.round(v * (1 << shift)), -(1 << (prec - 1)), (1 << (prec - 1)) - 1)) for v in c]
        for v in x[:o]:
            bw.put_signed(v, sb)
        bw.put(prec - 1, 4)
        bw.put_signed(shift, 5)
        for v in q:
            bw.put_signed(v, prec)
        res = []
        for n in range(o, block):
            res.append(x[n] - (sum(q[j] * x[n - 1 - j] for j in range(o)) >> shift))
        write_residual(bw, res, block, o, kw.get("method", 0), kw.get("porder"), kw.get("escape"))


RATE_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
              48000: 10, 96000: 11}
BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def block_code(n):
    table = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12, 8192: 13,
             16384: 14, 32768: 15}
    if n in table:
        return table[n], b""
    if n <= 256:
        return 6, bytes([n - 1])
    return 7, (n - 1).to_bytes(2, "big")


def rate_bits(rate, force0=False):
    if force0:
        return 0, b""
    if rate in RATE_CODES:
        return RATE_CODES[rate], b""
    if rate % 1000 == 0 and rate // 1000 < 256:
        return 12, bytes([rate // 1000])
    if rate < 65536:
        return 13, rate.to_bytes(2, "big")
    if rate % 10 == 0 and rate // 10 < 65536:
        return 14, (rate // 10).to_bytes(2, "big")
    return 0, b""


def encode(pcm, rate, bps, block=4096, variable=False, plan=None, stereo=None, force_codes0=False, seed=0):
    """pcm: int array (channels, n).  plan(frame_index, channel) -> (kind, kwargs) or None (auto)."""
    pcm = np.asarray(pcm, dtype=np.int64)
    ch, n = pcm.shape
    rng = np.random.default_rng(seed)
    frames = []
    start, fi = 0, 0
    min_b, max_b = 1 << 16, 0
    while start < n:
        bsz = min(block if not variable else int(rng.integers(block // 2, block + 1)), n - start)
        min_b, max_b = min(min_b, bsz), max(max_b, bsz)
        x = pcm[:, start:start + bsz]
        mode = stereo(fi) if (stereo is not None and ch == 2) else ch - 1
        hdr = BitWriter()
        hdr.put(0x3FFE, 14)
        hdr.put(0, 1)
        hdr.put(1 if variable else 0, 1)
        bc, bextra = block_code(bsz)
        rc, rextra = rate_bits(rate, force_codes0)
        hdr.put(bc, 4)
        hdr.put(rc, 4)
        hdr.put(mode, 4)
        hdr.put(0 if force_codes0 or bps not in BPS_CODES else BPS_CODES[bps], 3)
        hdr.put(0, 1)
        head = hdr.bytes() + utf8_num(start if variable else fi) + bextra + rextra
        head += bytes([crc8(head)])
        bw = BitWriter()
        if mode == 8:
            chans = [(x[0], bps), (x[0] - x[1], bps + 1)]
        elif mode == 9:
            chans = [(x[0] - x[1], bps + 1), (x[1], bps)]
        elif mode == 10:
            chans = [((x[0] + x[1]) >> 1, bps), (x[0] - x[1], bps + 1)]
        else:
            chans = [(x[c], bps) for c in range(ch)]
        for c, (v, b) in enumerate(chans):
            choice = plan(fi, c) if plan else None
            if choice is None:
                choice = ("constant", {}) if len(set(v.tolist())) == 1 else ("fixed", {"order": min(2, bsz)})
            kind, kw = choice
            write_subframe(bw, v, b, kind, **kw)
        bw.align()
        body = head + bw.bytes()
        frames.append(body + crc16(body).to_bytes(2, "big"))
        start += bsz
        fi += 1
    md5 = hashlib.md5()
    nbytes = (bps + 7) // 8
    inter = pcm.T.reshape(-1)
    md5.update(b"".join(int(v).to_bytes(nbytes, "little", signed=True) for v in inter))
    si = BitWriter()
    si.put(min_b if not variable else min(min_b, max_b), 16)
    si.put(max_b, 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(rate, 20)
    si.put(ch - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    info = si.bytes() + md5.digest()
    meta = bytes([0x00]) + len(info).to_bytes(3, "big") + info
    pad = bytes([0x81]) + (7).to_bytes(3, "big") + bytes(7)  # a last PADDING block
    return b"fLaC" + meta + pad + b"".join(frames)
