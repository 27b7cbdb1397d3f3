"""FLAC decoder for reference clips (host side, once per clip).

The reference reads reference audio with libsndfile (`soundfile.read(path,
dtype='float32')`, src/genie_tts/Audio/Audio.py:24) and accepts `.flac` clips
(src/genie_tts/Internal.py:38, Server.py:20).  Neither libsndfile nor any FLAC
tool exists in this image, so this module decodes the format itself, following
the published specification (RFC 9639): STREAMINFO, frame headers (fixed and
variable block sizes, coded sample rates / sizes), CONSTANT / VERBATIM / FIXED
(orders 0-4) / LPC (orders 1-32) subframes with wasted bits, Rice and Rice2
residuals with escape partitions, the four channel assignments, and the CRC-8
(header) / CRC-16 (frame) checks.  Decoding is lossless, so the integer samples
are exact; they are scaled to float32 the way libsndfile does (x / 2^(bits-1)).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


class FlacError(ValueError):
    pass


def _crc_table(poly: int, width: int):
    top, mask = 1 << (width - 1), (1 << width) - 1
    tab = []
    for b in range(256):
        c = b << (width - 8)
        for _ in range(8):
            c = ((c << 1) ^ poly) if c & top else (c << 1)
        tab.append(c & mask)
    return tab


_CRC8 = _crc_table(0x07, 8)
_CRC16 = _crc_table(0x8005, 16)


def crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c = _CRC8[c ^ b]
    return c


def crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c = ((c << 8) & 0xFFFF) ^ _CRC16[(c >> 8) ^ b]
    return c


class _Bits:
    """MSB-first bit reader over a bytes object."""

    def __init__(self, data: bytes, pos: int = 0):
        self.data = data
        self.bit = pos * 8
        self._bits = None   # lazily unpacked bit array (residual decoding)

    def read(self, n: int) -> int:
        if n == 0:
            return 0
        b0 = self.bit >> 3
        b1 = (self.bit + n + 7) >> 3
        if b1 > len(self.data):
            raise FlacError("truncated stream")
        v = int.from_bytes(self.data[b0:b1], "big")
        v >>= (b1 * 8 - self.bit - n)
        self.bit += n
        return v & ((1 << n) - 1)

    def read_signed(self, n: int) -> int:
        v = self.read(n)
        return v - (1 << n) if n and v >> (n - 1) else v

    def unary(self) -> int:   # zeros before the next 1 bit
        n = 0
        while self.read(1) == 0:
            n += 1
        return n

    def align(self) -> None:
        self.bit = (self.bit + 7) & ~7

    @property
    def byte(self) -> int:
        return self.bit >> 3

    def bits_array(self):
        if self._bits is None:
            self._bits = np.unpackbits(np.frombuffer(self.data, np.uint8))
            self._ones = np.flatnonzero(self._bits)
        return self._bits, self._ones


def _utf8_number(r: _Bits) -> int:
    b = r.read(8)
    if b < 0x80:
        return b
    n = 0
    while b & (0x80 >> n):
        n += 1
    if n < 2 or n > 7:
        raise FlacError("bad coded frame number")
    v = b & ((1 << (7 - n)) - 1) if n < 7 else 0
    for _ in range(n - 1):
        c = r.read(8)
        if c >> 6 != 2:
            raise FlacError("bad coded frame number")
        v = (v << 6) | (c & 0x3F)
    return v


def _rice_partition(r: _Bits, n: int, k: int) -> List[int]:
    """n Rice-coded (parameter k) zigzag residuals, starting at r's bit position."""
    bits, ones = r.bits_array()
    out = []
    p = r.bit
    for _ in range(n):
        i = int(np.searchsorted(ones, p))
        if i >= len(ones):
            raise FlacError("truncated residual")
        q = int(ones[i]) - p
        p = int(ones[i]) + 1
        low = 0
        if k:
            b0, b1 = p >> 3, (p + k + 7) >> 3
            low = (int.from_bytes(r.data[b0:b1], "big") >> (b1 * 8 - p - k)) & ((1 << k) - 1)
            p += k
        u = (q << k) | low
        out.append((u >> 1) ^ -(u & 1))
    r.bit = p
    return out


def _residual(r: _Bits, block: int, order: int) -> List[int]:
    method = r.read(2)
    if method > 1:
        raise FlacError("reserved residual coding method")
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    porder = r.read(4)
    if (block >> porder) < order or block % (1 << porder):
        raise FlacError("bad partition order")
    res: List[int] = []
    for p in range(1 << porder):
        n = (block >> porder) - (order if p == 0 else 0)
        k = r.read(pbits)
        if k == esc:
            nb = r.read(5)
            res += [r.read_signed(nb) if nb else 0 for _ in range(n)]
        else:
            res += _rice_partition(r, n, k)
    return res


_FIXED = {0: (), 1: (1,), 2: (2, -1), 3: (3, -3, 1), 4: (4, -6, 4, -1)}


def _subframe(r: _Bits, block: int, bps: int) -> List[int]:
    if r.read(1):
        raise FlacError("subframe padding bit set")
    t = r.read(6)
    wasted = 0
    if r.read(1):
        wasted = r.unary() + 1
        bps -= wasted
    if t == 0:                                   # CONSTANT
        x = [r.read_signed(bps)] * block
    elif t == 1:                                 # VERBATIM
        x = [r.read_signed(bps) for _ in range(block)]
    elif 8 <= t <= 12:                           # FIXED, order t - 8
        order = t - 8
        x = [r.read_signed(bps) for _ in range(order)]
        res = _residual(r, block, order)
        c = _FIXED[order]
        for e in res:
            s = e
            for j, cj in enumerate(c):
                s += cj * x[-1 - j]
            x.append(s)
    elif t >= 32:                                # LPC, order t - 31
        order = t - 31
        x = [r.read_signed(bps) for _ in range(order)]
        prec = r.read(4) + 1
        if prec == 16:
            raise FlacError("invalid LPC precision")
        shift = r.read_signed(5)
        if shift < 0:
            raise FlacError("negative LPC shift")
        coef = [r.read_signed(prec) for _ in range(order)]
        res = _residual(r, block, order)
        rc = coef[::-1]                          # rc[i] multiplies x[n - order + i]
        for e in res:
            acc = 0
            w = x[-order:]
            for cj, xj in zip(rc, w):
                acc += cj * xj
            x.append(e + (acc >> shift))
    else:
        raise FlacError(f"reserved subframe type {t}")
    if wasted:
        x = [v << wasted for v in x]
    return x


_RATES = {1: 88200, 2: 176400, 3: 192000, 4: 8000, 5: 16000, 6: 22050, 7: 24000, 8: 32000, 9: 44100,
          10: 48000, 11: 96000}
_SIZES = {1: 8, 2: 12, 4: 16, 5: 20, 6: 24, 7: 32}


def _next_sync(data: bytes, pos: int) -> int:
    """Byte offset of the next frame sync code (0xFFF8 / 0xFFF9) at or after pos, or -1."""
    while True:
        i = data.find(b"\xff", pos)
        if i < 0 or i + 1 >= len(data):
            return -1
        if data[i + 1] in (0xF8, 0xF9):
            return i
        pos = i + 1


def _frame(r: "_Bits", data: bytes, start: int, info: dict, rate: int):
    """One frame after its sync code -> (sample rate, bits per sample, channel samples)."""
    r.read(1)                                # blocking strategy (fixed / variable)
    bcode, rcode, chmode, scode = r.read(4), r.read(4), r.read(4), r.read(3)
    r.read(1)
    _utf8_number(r)
    if bcode == 0:
        raise FlacError("reserved block size")
    block = (192 if bcode == 1 else 576 << (bcode - 2) if bcode <= 5 else
             r.read(8) + 1 if bcode == 6 else r.read(16) + 1 if bcode == 7 else 256 << (bcode - 8))
    if rcode == 12:
        rate = r.read(8) * 1000
    elif rcode == 13:
        rate = r.read(16)
    elif rcode == 14:
        rate = r.read(16) * 10
    elif rcode == 15:
        raise FlacError("invalid sample rate code")
    elif rcode:
        rate = _RATES[rcode]
    fbps = info["bps"] if scode == 0 else _SIZES.get(scode)
    if fbps is None:
        raise FlacError("reserved sample size")
    hcrc = r.read(8)
    if crc8(data[start:r.byte - 1]) != hcrc:
        raise FlacError(f"frame header CRC mismatch at byte {start}")
    if chmode <= 7:
        n_ch = chmode + 1
        sub = [_subframe(r, block, fbps) for _ in range(n_ch)]
    elif chmode <= 10:
        n_ch = 2
        side_first = chmode == 9
        a = _subframe(r, block, fbps + (1 if side_first else 0))
        b = _subframe(r, block, fbps + (0 if side_first else 1))
        if chmode == 8:                      # left, side
            sub = [a, [l - s for l, s in zip(a, b)]]
        elif chmode == 9:                    # side, right
            sub = [[s + rr for s, rr in zip(a, b)], b]
        else:                                # mid, side
            left, right = [], []
            for m, s in zip(a, b):
                m = (m << 1) | (s & 1)
                left.append((m + s) >> 1)
                right.append((m - s) >> 1)
            sub = [left, right]
    else:
        raise FlacError("reserved channel assignment")
    if n_ch != info["channels"]:
        raise FlacError("channel count differs from STREAMINFO")
    r.align()
    fcrc = r.read(16)
    if crc16(data[start:r.byte - 2]) != fcrc:
        raise FlacError(f"frame CRC mismatch at byte {start}")
    return rate, fbps, sub


def decode(data: bytes) -> Tuple[np.ndarray, int, int]:
    """FLAC bytes -> (int32 samples [frames, channels], sample rate, bits per sample)."""
    if data[:4] != b"fLaC":
        raise FlacError("not a FLAC stream")
    pos, info = 4, None
    while True:
        if pos + 4 > len(data):
            raise FlacError("truncated metadata")
        hdr = data[pos]
        last, btype = hdr >> 7, hdr & 0x7F
        length = int.from_bytes(data[pos + 1:pos + 4], "big")
        body = data[pos + 4:pos + 4 + length]
        if btype == 0:
            r = _Bits(body)
            r.read(16); r.read(16); r.read(24); r.read(24)
            info = dict(rate=r.read(20), channels=r.read(3) + 1, bps=r.read(5) + 1, total=r.read(36))
        pos += 4 + length
        if last:
            break
    if info is None:
        raise FlacError("missing STREAMINFO")
    chans: List[List[int]] = [[] for _ in range(info["channels"])]
    r = _Bits(data, pos)
    rate, bps = info["rate"], info["bps"]
    while r.byte + 2 <= len(data):
        if info["total"] and len(chans[0]) >= info["total"]:
            break                                # every sample STREAMINFO announced: trailing
                                                 # bytes (an ID3v1 'TAG' block, padding) are not audio
        start = r.byte
        try:
            if r.read(15) != 0x7FFC:             # sync 0b11111111111110 + reserved 0
                raise FlacError(f"lost frame sync at byte {start}")
            rate, bps, sub = _frame(r, data, start, info, rate)
        except FlacError:
            if not chans[0]:
                raise
            # after audio: bytes that are no frame (a tag, padding, junk holding a sync code);
            # libFLAC searches for the next frame, so do we
            nxt = _next_sync(data, start + 1)
            if nxt < 0:
                break
            r = _Bits(data, nxt)
            continue
        for c, x in zip(chans, sub):
            c.extend(x)
    if info["total"] and len(chans[0]) < info["total"]:
        raise FlacError(f"{len(chans[0])} samples decoded, STREAMINFO announces {info['total']}")
    pcm = np.asarray(chans, np.int64).T
    if info["total"]:
        pcm = pcm[:info["total"]]
    return pcm.astype(np.int32), rate, bps


def read_flac(path: str) -> Tuple[np.ndarray, int]:
    """-> (float32 [frames, channels], sample rate), scaled like libsndfile's float read."""
    with open(path, "rb") as f:
        pcm, rate, bps = decode(f.read())
    return (pcm.astype(np.float64) / float(1 << (bps - 1))).astype(np.float32), rate
