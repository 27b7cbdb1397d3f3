"""Minimal FLAC encoder for tests (RFC 9639), written independently of the decoder in
genie_tts_amd/flac.py so the two check each other: every subframe type (CONSTANT,
VERBATIM, FIXED orders 0-4, LPC with a given quantised predictor), wasted bits, Rice /
Rice2 residuals with partitions and escape partitions, every stereo channel
assignment, fixed or variable block sizes, coded and STREAMINFO sample rates / sizes."""
from __future__ import annotations

import numpy as np

from genie_tts_amd.flac import crc8, crc16


class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v: int, n: int):
        for i in range(n - 1, -1, -1):
            self.bits.append((v >> i) & 1)

    def put_signed(self, v: int, n: int):
        self.put(v & ((1 << n) - 1), n)

    def unary(self, q: int):
        self.bits += [0] * q + [1]

    def align(self):
        while len(self.bits) % 8:
            self.bits.append(0)

    def bytes(self) -> bytes:
        assert len(self.bits) % 8 == 0
        return np.packbits(np.asarray(self.bits, np.uint8)).tobytes()


def _utf8(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    for nb in range(2, 8):
        if n < 1 << (5 * nb + 1):
            break
    out = []
    for _ in range(nb - 1):
        out.append(0x80 | (n & 0x3F))
        n >>= 6
    first = ((0xFF00 >> nb) & 0xFF) | n
    return bytes([first] + out[::-1])


def _zigzag(e: int) -> int:
    return (e << 1) if e >= 0 else ((-e << 1) - 1)


def _residual(w: BitWriter, res, porder: int, rice2: bool, escape_first: bool, order: int, block: int):
    w.put(1 if rice2 else 0, 2)
    w.put(porder, 4)
    pbits, esc = (5, 31) if rice2 else (4, 15)
    i = 0
    for p in range(1 << porder):
        n = (block >> porder) - (order if p == 0 else 0)
        part = res[i:i + n]
        i += n
        if escape_first and p == 0:
            nb = max([abs(int(e)).bit_length() + 1 for e in part] + [0])
            w.put(esc, pbits)
            w.put(nb, 5)
            for e in part:
                if nb:
                    w.put_signed(int(e), nb)
            continue
        mean = np.mean([_zigzag(int(e)) for e in part]) if len(part) else 0
        k = max(0, min(esc - 1, int(np.log2(mean + 1)) if mean > 0 else 0))
        w.put(k, pbits)
        for e in part:
            u = _zigzag(int(e))
            w.unary(u >> k)
            if k:
                w.put(u & ((1 << k) - 1), k)


FIXED = {0: (), 1: (1,), 2: (2, -1), 3: (3, -3, 1), 4: (4, -6, 4, -1)}


def _subframe(w: BitWriter, x, bps: int, kind: str, wasted: int = 0, **kw):
    x = [int(v) for v in x]
    block = len(x)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in x)
        x = [v >> wasted for v in x]
        bps -= wasted
    code = {"constant": 0, "verbatim": 1}.get(kind)
    if kind == "fixed":
        code = 8 + kw["order"]
    elif kind == "lpc":
        code = 31 + len(kw["coef"])
    w.put(0, 1)
    w.put(code, 6)
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)
    if kind == "constant":
        assert len(set(x)) == 1
        w.put_signed(x[0], bps)
        return
    if kind == "verbatim":
        for v in x:
            w.put_signed(v, bps)
        return
    porder, rice2, esc = kw.get("porder", 0), kw.get("rice2", False), kw.get("escape", False)
    if kind == "fixed":
        order = kw["order"]
        c = FIXED[order]
        res = [x[n] - sum(cj * x[n - 1 - j] for j, cj in enumerate(c)) for n in range(order, block)]
        for v in x[:order]:
            w.put_signed(v, bps)
        _residual(w, res, porder, rice2, esc, order, block)
        return
    coef, shift, prec = kw["coef"], kw["shift"], kw["prec"]
    order = len(coef)
    res = [x[n] - (sum(coef[j] * x[n - 1 - j] for j in range(order)) >> shift) for n in range(order, block)]
    for v in x[:order]:
        w.put_signed(v, bps)
    w.put(prec - 1, 4)
    w.put_signed(shift, 5)
    for c in coef:
        w.put_signed(c, prec)
    _residual(w, res, porder, rice2, esc, order, block)


def encode(pcm: np.ndarray, rate: int, bps: int, frames, variable: bool = False, header_rate: bool = False,
           header_size: bool = True) -> bytes:
    """pcm int [n, channels]; frames = list of dicts: {"n": samples, "mode": chmode (0..10),
    "sub": [subframe kwargs per channel]} covering pcm in order."""
    n_total, nch = pcm.shape
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.put(16, 16); si.put(65535, 16); si.put(0, 24); si.put(0, 24)
    si.put(rate, 20); si.put(nch - 1, 3); si.put(bps - 1, 5); si.put(n_total, 36)
    si.put(0, 128)
    body = si.bytes()
    out += bytes([0x80 | 0]) + len(body).to_bytes(3, "big") + body
    pos, fno = 0, 0
    size_codes = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}
    for fr in frames:
        n = fr["n"]
        x = pcm[pos:pos + n].astype(np.int64)
        w = BitWriter()
        w.put(0x3FFE, 14); w.put(0, 1); w.put(1 if variable else 0, 1)
        bcode = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12}.get(n)
        if bcode is None:
            bcode = 6 if n <= 256 else 7
        w.put(bcode, 4)
        rcodes = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
                  48000: 10, 96000: 11}
        if header_rate:
            rcode = rcodes.get(rate, 13 if rate < 65536 else 12)
        else:
            rcode = 0
        w.put(rcode, 4)
        w.put(fr["mode"], 4)
        w.put(size_codes[bps] if header_size else 0, 3)
        w.put(0, 1)
        for b in _utf8(pos if variable else fno):
            w.put(b, 8)
        if bcode == 6:
            w.put(n - 1, 8)
        elif bcode == 7:
            w.put(n - 1, 16)
        if rcode == 13:
            w.put(rate, 16)
        elif rcode == 12:
            w.put(rate // 1000, 8)
        hdr = w.bytes()
        w.put(crc8(hdr), 8)
        mode = fr["mode"]
        if mode <= 7:
            chans = [(x[:, c], bps) for c in range(nch)]
        else:
            L, R = x[:, 0], x[:, 1]
            S = L - R
            if mode == 8:
                chans = [(L, bps), (S, bps + 1)]
            elif mode == 9:
                chans = [(S, bps + 1), (R, bps)]
            else:
                chans = [((L + R) >> 1, bps), (S, bps + 1)]
        for (xc, b), kw in zip(chans, fr["sub"]):
            _subframe(w, xc, b, **kw)
        w.align()
        data = w.bytes()
        out += data + crc16(data).to_bytes(2, "big")
        pos += n
        fno += 1
    assert pos == n_total
    return bytes(out)
