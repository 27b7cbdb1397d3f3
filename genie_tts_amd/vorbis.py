"""Ogg/Vorbis reader for reference clips.

The reference reads reference clips through libsndfile (`Audio/Audio.py:24`), which
accepts '.ogg' (`Internal.py:38`).  This module restates the published Vorbis I
specification (Xiph.Org, "Vorbis I specification") and the Ogg framing (RFC 3533):

  * Ogg pages (capture pattern, lacing, CRC-32 poly 0x04C11DB7) -> packets of the first
    Vorbis logical stream;
  * identification / comment / setup headers: codebooks (ordered and sparse codeword
    lengths, Huffman assignment in entry order, lookup types 1 and 2), floors 0 and 1,
    residues 0, 1 and 2, mappings (submaps, channel coupling), modes;
  * audio packets: floor decode and curve synthesis, residue VQ decode, inverse
    coupling, floor x residue, inverse MDCT (unnormalised, as libvorbis), the
    power-complementary Vorbis window with short/long transitions, overlap-add;
    samples per packet = previous blocksize / 4 + current blocksize / 4, the stream
    trimmed to the last page's granule position.

Output: float32 [frames, channels] in [-1, 1] (libsndfile's float read of a Vorbis file
is the decoder's float output).  Host code, numpy; a reference clip is seconds long.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np


class VorbisError(ValueError):
    pass


class _EndOfPacket(Exception):
    pass


# ------------------------------------------------------------------ Ogg
def _crc_table():
    t = []
    for i in range(256):
        r = i << 24
        for _ in range(8):
            r = ((r << 1) ^ 0x04C11DB7) & 0xFFFFFFFF if r & 0x80000000 else (r << 1) & 0xFFFFFFFF
        t.append(r)
    return t


_CRC = _crc_table()


def ogg_crc(data: bytes) -> int:
    c = 0
    for b in data:
        c = ((c << 8) & 0xFFFFFFFF) ^ _CRC[((c >> 24) ^ b) & 0xFF]
    return c


def ogg_packets(data: bytes) -> Tuple[List[bytes], int]:
    """Packets of the first logical stream and the last granule position seen."""
    pos, serial, packets, cur, last_gp = 0, None, [], b"", -1
    while pos < len(data):
        if data[pos:pos + 4] != b"OggS":
            raise VorbisError(f"lost Ogg capture pattern at byte {pos}")
        if pos + 27 > len(data):
            raise VorbisError("truncated Ogg page header")
        if data[pos + 4] != 0:
            raise VorbisError("unsupported Ogg version")
        htype = data[pos + 5]
        gp = int.from_bytes(data[pos + 6:pos + 14], "little", signed=True)
        sno = int.from_bytes(data[pos + 14:pos + 18], "little")
        crc = int.from_bytes(data[pos + 22:pos + 26], "little")
        nseg = data[pos + 26]
        lace = data[pos + 27:pos + 27 + nseg]
        body_len = sum(lace)
        end = pos + 27 + nseg + body_len
        if end > len(data):
            raise VorbisError("truncated Ogg page")
        page = bytearray(data[pos:end])
        page[22:26] = b"\0\0\0\0"
        if ogg_crc(bytes(page)) != crc:
            raise VorbisError(f"Ogg page CRC mismatch at byte {pos}")
        if serial is None:
            serial = sno
        if sno == serial:
            if not (htype & 1) and cur:
                raise VorbisError("Ogg packet continuation missing")
            off = pos + 27 + nseg
            for ln in lace:
                cur += data[off:off + ln]
                off += ln
                if ln < 255:
                    packets.append(cur)
                    cur = b""
            if gp != -1:
                last_gp = gp
        pos = end
    return packets, last_gp


# ------------------------------------------------------------------ bits
class _Bits:
    """LSb-first bit reader over one packet (Vorbis I section 2)."""

    def __init__(self, data: bytes):
        self.d = data
        self.n = len(data) * 8
        self.p = 0

    def read(self, k: int) -> int:
        if k == 0:
            return 0
        if self.p + k > self.n:
            self.p = self.n
            raise _EndOfPacket()
        v, got, p = 0, 0, self.p
        while got < k:
            byte = self.d[p >> 3]
            sh = p & 7
            take = min(8 - sh, k - got)
            v |= ((byte >> sh) & ((1 << take) - 1)) << got
            got += take
            p += take
        self.p = p
        return v

    def bit(self) -> int:
        if self.p >= self.n:
            raise _EndOfPacket()
        b = (self.d[self.p >> 3] >> (self.p & 7)) & 1
        self.p += 1
        return b

    def peek(self, k: int) -> int:
        """The next k bits (LSb-first, as read() would return them) without consuming
        them; bits past the end read as 0."""
        p = self.p
        b = p >> 3
        return (int.from_bytes(self.d[b:b + ((p & 7) + k + 7) // 8], "little") >> (p & 7)) & ((1 << k) - 1)


def ilog(x: int) -> int:
    return 0 if x <= 0 else x.bit_length()


def float32_unpack(x: int) -> float:
    mant = x & 0x1FFFFF
    exp = (x & 0x7FE00000) >> 21
    if x & 0x80000000:
        mant = -mant
    return math.ldexp(float(mant), exp - 788)


def lookup1_values(entries: int, dims: int) -> int:
    r = int(math.floor(entries ** (1.0 / dims)))
    while (r + 1) ** dims <= entries:
        r += 1
    while r ** dims > entries:
        r -= 1
    return r


# ------------------------------------------------------------------ codebooks
class Codebook:
    def __init__(self, r: _Bits):
        if r.read(24) != 0x564342:
            raise VorbisError("bad codebook sync pattern")
        self.dims = r.read(16)
        self.entries = r.read(24)
        lengths = [0] * self.entries
        if r.read(1):                                   # ordered
            cur_len = r.read(5) + 1
            i = 0
            while i < self.entries:
                num = r.read(ilog(self.entries - i))
                if i + num > self.entries:
                    raise VorbisError("codebook lengths overflow")
                for j in range(i, i + num):
                    lengths[j] = cur_len
                i += num
                cur_len += 1
        else:
            sparse = r.read(1)
            for i in range(self.entries):
                if not sparse or r.read(1):
                    lengths[i] = r.read(5) + 1
        self.lengths = lengths
        self.codes = self._assign(lengths)
        self._table()
        self.lookup_type = r.read(4)
        self.vq: Optional[np.ndarray] = None
        if self.lookup_type in (1, 2):
            mn = float32_unpack(r.read(32))
            delta = float32_unpack(r.read(32))
            bits = r.read(4) + 1
            seq = r.read(1)
            nval = lookup1_values(self.entries, self.dims) if self.lookup_type == 1 else self.entries * self.dims
            mult = [r.read(bits) for _ in range(nval)]
            vq = np.zeros((self.entries, self.dims), np.float32)
            for e in range(self.entries):
                last, div = 0.0, 1
                for d in range(self.dims):
                    off = (e // div) % nval if self.lookup_type == 1 else e * self.dims + d
                    v = mult[off] * delta + mn + last
                    if seq:
                        last = v
                    vq[e, d] = v
                    if self.lookup_type == 1:
                        div *= nval
            self.vq = vq
        elif self.lookup_type != 0:
            raise VorbisError(f"codebook lookup type {self.lookup_type}")

    @staticmethod
    def _assign(lengths: List[int]) -> Dict[Tuple[int, int], int]:
        """Huffman codewords in entry order: each entry takes the lowest codeword of its
        length still free (the spec's 'next available' rule), MSb = first bit read."""
        used = [(i, l) for i, l in enumerate(lengths) if l > 0]
        codes: Dict[Tuple[int, int], int] = {}
        if len(used) == 1:                              # a single used entry: one bit, either value
            codes[(0, 0)] = used[0][0]                  # (libvorbis: a 1-bit first table, both halves)
            return codes
        marker = [0] * 33
        for i, ln in used:
            entry = marker[ln]
            if ln < 32 and (entry >> ln):
                raise VorbisError("codebook is overspecified")
            codes[(ln, entry)] = i
            for j in range(ln, 0, -1):
                if marker[j] & 1:
                    marker[j] = marker[j - 1] << 1 if j > 1 else marker[j] + 1
                    break
                marker[j] += 1
            for j in range(ln + 1, 33):
                if (marker[j] >> 1) == entry:
                    entry = marker[j]
                    marker[j] = marker[j - 1] << 1
                else:
                    break
        return codes

    TABLE_BITS = 12

    def _table(self):
        """Direct lookup of codewords up to TABLE_BITS long: index = the next TABLE_BITS
        bits as read (the first bit read = the codeword's MSb = index bit 0); longer ones
        fall back to the bit-serial walk."""
        n = self.TABLE_BITS
        self._ent = [-1] * (1 << n)
        self._len = [0] * (1 << n)
        if (0, 0) in self.codes:
            return
        for (ln, code), e in self.codes.items():
            if ln > n:
                continue
            rev = int(format(code, f"0{ln}b")[::-1], 2)   # reading order -> LSb-first
            for hi in range(1 << (n - ln)):
                idx = rev | (hi << ln)
                self._ent[idx] = e
                self._len[idx] = ln

    def decode(self, r: _Bits) -> int:
        if (0, 0) in self.codes:
            r.bit()
            return self.codes[(0, 0)]
        idx = r.peek(self.TABLE_BITS)
        ln = self._len[idx]
        if ln and r.p + ln <= r.n:
            r.p += ln
            return self._ent[idx]
        code = 0
        for ln in range(1, 33):
            code = (code << 1) | r.bit()
            e = self.codes.get((ln, code))
            if e is not None:
                return e
        raise VorbisError("undecodable codeword")

    def decode_vq(self, r: _Bits) -> np.ndarray:
        if self.vq is None:
            raise VorbisError("VQ decode from a codebook without a lookup")
        return self.vq[self.decode(r)]


# ------------------------------------------------------------------ floors
# floor1_inverse_dB_table: 256 steps of 140/256 dB up to 1.0 (the spec's table,
# 1.0649863e-07 ... 1.0)
_INV_DB = np.array([10.0 ** ((i - 255) * 7.0 / 256.0) for i in range(256)], np.float32)
_F1_RANGE = (256, 128, 86, 64)


def _render_point(x0, y0, x1, y1, x):
    dy = y1 - y0
    adx = x1 - x0
    err = abs(dy) * (x - x0)
    off = err // adx
    return y0 - off if dy < 0 else y0 + off


def _render_line(x0, y0, x1, y1, v, n):
    dy = y1 - y0
    adx = x1 - x0
    base = int(dy / adx)                                # truncation toward zero
    sy = base - 1 if dy < 0 else base + 1
    ady = abs(dy) - abs(base) * adx
    x, y, err = x0, y0, 0
    if x < n:
        v[x] = y
    for x in range(x0 + 1, min(x1, n)):
        err += ady
        if err >= adx:
            err -= adx
            y += sy
        else:
            y += base
        v[x] = y


class Floor1:
    def __init__(self, r: _Bits):
        npart = r.read(5)
        self.part_class = [r.read(4) for _ in range(npart)]
        maxc = max(self.part_class) if npart else -1
        self.cdim, self.csub, self.cmaster, self.subbooks = [], [], [], []
        for _ in range(maxc + 1):
            self.cdim.append(r.read(3) + 1)
            sub = r.read(2)
            self.csub.append(sub)
            self.cmaster.append(r.read(8) if sub else -1)
            self.subbooks.append([r.read(8) - 1 for _ in range(1 << sub)])
        self.mult = r.read(2) + 1
        rb = r.read(4)
        self.xs = [0, 1 << rb]
        for c in self.part_class:
            for _ in range(self.cdim[c]):
                self.xs.append(r.read(rb))
        if len(set(self.xs)) != len(self.xs):
            raise VorbisError("floor1 X values repeat")
        # neighbours of each point among the earlier ones
        self.lo, self.hi = [0, 0], [0, 0]
        for i in range(2, len(self.xs)):
            x = self.xs[i]
            lo = max((j for j in range(i) if self.xs[j] < x), key=lambda j: self.xs[j])
            hi = min((j for j in range(i) if self.xs[j] > x), key=lambda j: self.xs[j])
            self.lo.append(lo)
            self.hi.append(hi)

    def decode(self, r: _Bits, books: List[Codebook]):
        if not r.read(1):
            return None
        rng = _F1_RANGE[self.mult - 1]
        y = [r.read(ilog(rng - 1)), r.read(ilog(rng - 1))]
        for c in self.part_class:
            cbits = self.csub[c]
            cval = books[self.cmaster[c]].decode(r) if cbits else 0
            for _ in range(self.cdim[c]):
                book = self.subbooks[c][cval & ((1 << cbits) - 1)]
                cval >>= cbits
                y.append(books[book].decode(r) if book >= 0 else 0)
        return y

    def curve(self, y: List[int], n2: int) -> np.ndarray:
        rng = _F1_RANGE[self.mult - 1]
        m = len(self.xs)
        final = list(y[:2]) + [0] * (m - 2)
        step2 = [True, True] + [False] * (m - 2)
        for i in range(2, m):
            lo, hi = self.lo[i], self.hi[i]
            pred = _render_point(self.xs[lo], final[lo], self.xs[hi], final[hi], self.xs[i])
            val = y[i]
            highroom, lowroom = rng - pred, pred
            room = 2 * (highroom if highroom < lowroom else lowroom)
            if val:
                step2[lo] = step2[hi] = step2[i] = True
                if val >= room:
                    final[i] = val - lowroom + pred if highroom > lowroom else pred - val + highroom - 1
                else:
                    final[i] = pred - (val + 1) // 2 if val & 1 else pred + val // 2
            else:
                final[i] = pred
        order = sorted(range(m), key=lambda i: self.xs[i])
        v = np.zeros(n2, np.int64)
        lx, ly, hx, hy = 0, final[order[0]] * self.mult, 0, 0
        for i in order[1:]:
            if step2[i]:
                hy = final[i] * self.mult
                hx = self.xs[i]
                _render_line(lx, ly, hx, hy, v, n2)
                lx, ly = hx, hy
        if hx < n2:
            _render_line(hx, hy, n2, hy, v, n2)
        return _INV_DB[np.clip(v, 0, 255)]


class Floor0:
    def __init__(self, r: _Bits):
        self.order = r.read(8)
        self.rate = r.read(16)
        self.bark_size = r.read(16)
        self.amp_bits = r.read(6)
        self.amp_off = r.read(8)
        self.books = [r.read(8) for _ in range(r.read(4) + 1)]

    def decode(self, r: _Bits, books: List[Codebook]):
        amp = r.read(self.amp_bits)
        if amp == 0:
            return None
        bn = r.read(ilog(len(self.books)))
        if bn >= len(self.books):
            raise VorbisError("floor0 book number")
        book = books[self.books[bn]]
        coef: List[float] = []
        last = 0.0
        while len(coef) < self.order:
            v = book.decode_vq(r).astype(np.float64) + last
            coef.extend(v.tolist())
            last = coef[-1]
        return amp, coef[:self.order]

    def curve(self, dec, n2: int) -> np.ndarray:
        amp, coef = dec

        def bark(x):
            return 13.1 * math.atan(0.00074 * x) + 2.24 * math.atan(0.0000000185 * x * x) + 0.0001 * x
        scale = self.bark_size / bark(0.5 * self.rate)
        out = np.zeros(n2, np.float32)
        cosc = [math.cos(c) for c in coef]
        i = 0
        while i < n2:
            mi = min(self.bark_size - 1, int(math.floor(bark(self.rate * i / (2.0 * n2)) * scale)))
            w = math.pi * mi / self.bark_size
            cw = math.cos(w)
            o = self.order
            if o & 1:
                p = (1 - cw * cw) * np.prod([4 * (cosc[2 * j + 1] - cw) ** 2 for j in range((o - 3) // 2 + 1)])
                q = 0.25 * np.prod([4 * (cosc[2 * j] - cw) ** 2 for j in range((o - 1) // 2 + 1)])
            else:
                p = (1 - cw) / 2 * np.prod([4 * (cosc[2 * j + 1] - cw) ** 2 for j in range((o - 2) // 2 + 1)])
                q = (1 + cw) / 2 * np.prod([4 * (cosc[2 * j] - cw) ** 2 for j in range((o - 2) // 2 + 1)])
            pq = math.sqrt(p + q)
            ex = 0.11512925 * (amp * self.amp_off / (((1 << self.amp_bits) - 1) * pq) - self.amp_off) if pq > 0 \
                else math.inf
            val = math.exp(ex) if ex < 709.0 else math.inf   # beyond the double range: inf, as a float curve
            while i < n2:                                # every i with the same map value
                out[i] = val
                i += 1
                if i < n2 and min(self.bark_size - 1,
                                  int(math.floor(bark(self.rate * i / (2.0 * n2)) * scale))) != mi:
                    break
        return out


# ------------------------------------------------------------------ residues
class Residue:
    def __init__(self, r: _Bits, rtype: int):
        self.type = rtype
        self.begin = r.read(24)
        self.end = r.read(24)
        self.psize = r.read(24) + 1
        self.nclass = r.read(6) + 1
        self.classbook = r.read(8)
        casc = []
        for _ in range(self.nclass):
            low = r.read(3)
            high = r.read(5) if r.read(1) else 0
            casc.append(high * 8 + low)
        self.books = [[r.read(8) if (c >> j) & 1 else -1 for j in range(8)] for c in casc]

    def decode(self, r: _Bits, books: List[Codebook], nvec: int, n2: int, skip: List[bool]) -> List[np.ndarray]:
        if self.type == 2:
            out = [np.zeros(n2, np.float32) for _ in range(nvec)]
            if all(skip):
                return out
            v = self._decode(r, books, [np.zeros(n2 * nvec, np.float32)], n2 * nvec, [False])[0]
            for c in range(nvec):
                out[c] = v[c::nvec].copy()
            return out
        vecs = [np.zeros(n2, np.float32) for _ in range(nvec)]
        return self._decode(r, books, vecs, n2, skip)

    def _decode(self, r, books, vecs, size, skip):
        cb = books[self.classbook]
        lb, le = min(self.begin, size), min(self.end, size)
        nparts = (le - lb) // self.psize
        cpw = cb.dims
        classes = [[0] * (nparts + cpw) for _ in vecs]
        fmt0 = self.type == 0
        try:
            for pss in range(8):
                pc = 0
                while pc < nparts:
                    if pss == 0:
                        for j in range(len(vecs)):
                            if skip[j]:
                                continue
                            temp = cb.decode(r)
                            for i in range(cpw - 1, -1, -1):
                                classes[j][i + pc] = temp % self.nclass
                                temp //= self.nclass
                    for _ in range(cpw):
                        if pc >= nparts:
                            break
                        for j, v in enumerate(vecs):
                            if skip[j]:
                                continue
                            bk = self.books[classes[j][pc]][pss]
                            if bk < 0:
                                continue
                            book = books[bk]
                            off = lb + pc * self.psize
                            if fmt0:
                                step = self.psize // book.dims
                                for i in range(step):
                                    e = book.decode_vq(r)
                                    v[off + i: off + i + step * book.dims: step] += e
                            else:
                                i = 0
                                while i < self.psize:
                                    e = book.decode_vq(r)
                                    v[off + i: off + i + book.dims] += e
                                    i += book.dims
                        pc += 1
        except _EndOfPacket:
            pass                                          # the rest of the vectors stays zero
        return vecs


# ------------------------------------------------------------------ transform
def imdct(X: np.ndarray) -> np.ndarray:
    """y[i] = sum_k X[k] cos(pi / (2N) (2i + 1 + N/2)(2k + 1)), N = 2 len(X), i < N (no
    scaling, as libvorbis).  With n0 = N/4 + 1/2 the sum is
    Re(e^{i pi (i + n0) / N} sum_k X[k] e^{i 2 pi n0 k / N} e^{i 2 pi i k / N}): one N-point
    inverse FFT of the twiddled, zero-padded coefficients, in float64."""
    x = np.asarray(X, np.float64)
    M = x.shape[0]
    N = 2 * M
    n0 = N / 4.0 + 0.5
    z = np.zeros(N, np.complex128)
    k = np.arange(M)
    z[:M] = x * np.exp(2j * np.pi * n0 * k / N)
    s = np.fft.ifft(z) * N
    i = np.arange(N)
    return (np.exp(1j * np.pi * (i + n0) / N) * s).real


def window(n: int, bs0: int, long_block: bool, prev_long: bool, next_long: bool) -> np.ndarray:
    w = np.zeros(n)
    center = n // 2
    if long_block and not prev_long:
        ls, le, ln = n // 4 - bs0 // 4, n // 4 + bs0 // 4, bs0 // 2
    else:
        ls, le, ln = 0, center, n // 2
    if long_block and not next_long:
        rs, re_, rn = n * 3 // 4 - bs0 // 4, n * 3 // 4 + bs0 // 4, bs0 // 2
    else:
        rs, re_, rn = center, n, n // 2
    i = np.arange(ls, le)
    w[ls:le] = np.sin(np.pi / 2 * np.sin((i - ls + 0.5) / ln * np.pi / 2) ** 2)
    w[le:rs] = 1.0
    i = np.arange(rs, re_)
    w[rs:re_] = np.sin(np.pi / 2 * np.sin((i - rs + 0.5) / rn * np.pi / 2 + np.pi / 2) ** 2)
    return w


# ------------------------------------------------------------------ decoder
class VorbisDecoder:
    def __init__(self, packets: List[bytes]):
        if len(packets) < 3:
            raise VorbisError("missing Vorbis headers")
        self._ident(packets[0])
        self._comment(packets[1])
        self._setup(packets[2])
        self.audio = packets[3:]

    @staticmethod
    def _hdr(p: bytes, t: int) -> _Bits:
        if len(p) < 7 or p[0] != t or p[1:7] != b"vorbis":
            raise VorbisError(f"expected Vorbis header type {t}")
        r = _Bits(p)
        r.p = 7 * 8
        return r

    def _ident(self, p: bytes):
        r = self._hdr(p, 1)
        if r.read(32) != 0:
            raise VorbisError("unsupported Vorbis version")
        self.channels = r.read(8)
        self.rate = r.read(32)
        r.read(32); r.read(32); r.read(32)
        self.bs0 = 1 << r.read(4)
        self.bs1 = 1 << r.read(4)
        if not r.read(1) or self.channels == 0 or self.rate == 0 or not (64 <= self.bs0 <= self.bs1 <= 8192):
            raise VorbisError("bad identification header")

    def _comment(self, p: bytes):
        self._hdr(p, 3)                                   # vendor / user comments: not needed

    def _setup(self, p: bytes):
        r = self._hdr(p, 5)
        try:
            self.books = [Codebook(r) for _ in range(r.read(8) + 1)]
            for _ in range(r.read(6) + 1):
                if r.read(16) != 0:
                    raise VorbisError("time domain transform")
            self.floors = []
            for _ in range(r.read(6) + 1):
                t = r.read(16)
                if t == 0:
                    self.floors.append(Floor0(r))
                elif t == 1:
                    self.floors.append(Floor1(r))
                else:
                    raise VorbisError(f"floor type {t}")
            self.residues = []
            for _ in range(r.read(6) + 1):
                t = r.read(16)
                if t > 2:
                    raise VorbisError(f"residue type {t}")
                self.residues.append(Residue(r, t))
            self.mappings = []
            for _ in range(r.read(6) + 1):
                if r.read(16) != 0:
                    raise VorbisError("mapping type")
                subs = r.read(4) + 1 if r.read(1) else 1
                coupling = []
                if r.read(1):
                    for _ in range(r.read(8) + 1):
                        coupling.append((r.read(ilog(self.channels - 1)), r.read(ilog(self.channels - 1))))
                if r.read(2) != 0:
                    raise VorbisError("mapping reserved bits")
                mux = [r.read(4) for _ in range(self.channels)] if subs > 1 else [0] * self.channels
                sub = []
                for _ in range(subs):
                    r.read(8)
                    sub.append((r.read(8), r.read(8)))
                self.mappings.append((coupling, mux, sub))
            self.modes = []
            for _ in range(r.read(6) + 1):
                bf = r.read(1)
                if r.read(16) != 0 or r.read(16) != 0:
                    raise VorbisError("mode window / transform type")
                self.modes.append((bf, r.read(8)))
            if not r.read(1):
                raise VorbisError("setup framing bit")
        except _EndOfPacket:
            raise VorbisError("truncated setup header") from None

    def decode(self) -> np.ndarray:
        out = np.zeros((0, self.channels))
        buf: Optional[np.ndarray] = None                    # previous frame's windowed output
        prev_n = 0
        chunks = []
        for pk in self.audio:
            frame = self._packet(pk)
            if frame is None:
                continue
            y, n = frame
            if buf is not None:
                # overlap: the previous frame's right half with this frame's left half; the
                # samples from the previous centre to this centre are complete
                a = prev_n // 4 + n // 4
                seg = np.zeros((a, self.channels))
                p0 = prev_n // 2                             # previous centre in its own frame
                s0 = prev_n // 4 + prev_n // 2 - n // 4      # this frame's start in the previous frame
                # previous contribution: its samples [p0, prev_n) land at seg[0: prev_n - p0]
                prev_part = buf[p0:]
                seg[:min(a, prev_part.shape[0])] += prev_part[:a]
                # this frame's samples [0, n/2) land at seg[s0 - p0 : ...]
                off = s0 - p0
                cur = y[:n // 2]
                lo = max(0, -off)
                hi = min(n // 2, a - off)
                if hi > lo:
                    seg[off + lo: off + hi] += cur[lo:hi]
                chunks.append(seg)
            buf = y
            prev_n = n
        if chunks:
            out = np.concatenate(chunks, axis=0)
        return out

    def _packet(self, pk: bytes):
        r = _Bits(pk)
        try:
            if r.read(1) != 0:
                return None                                # not an audio packet
            mode = r.read(ilog(len(self.modes) - 1))
            if mode >= len(self.modes):
                raise VorbisError("mode number")
            bf, mapping = self.modes[mode]
            n = self.bs1 if bf else self.bs0
            prev_long = next_long = True
            if bf:
                prev_long, next_long = bool(r.read(1)), bool(r.read(1))
        except _EndOfPacket:
            return None
        n2 = n // 2
        coupling, mux, subs = self.mappings[mapping]
        ch = self.channels
        floors: List = [None] * ch
        try:
            for c in range(ch):
                fl = self.floors[subs[mux[c]][0]]
                d = fl.decode(r, self.books)
                floors[c] = None if d is None else (fl, d)
        except _EndOfPacket:
            floors = [None] * ch
        nonzero = [f is not None for f in floors]
        for m, a in coupling:
            if nonzero[m] or nonzero[a]:
                nonzero[m] = nonzero[a] = True
        res = [np.zeros(n2, np.float32) for _ in range(ch)]
        for si, (_, rn) in enumerate(subs):
            chans = [c for c in range(ch) if mux[c] == si]
            vecs = self.residues[rn].decode(r, self.books, len(chans), n2, [not nonzero[c] for c in chans])
            for c, v in zip(chans, vecs):
                res[c] = v
        for m, a in reversed(coupling):
            M, A = res[m].astype(np.float32), res[a].astype(np.float32)
            pos_m, pos_a = M > 0, A > 0
            newM = np.where(pos_m, np.where(pos_a, M, M + A), np.where(pos_a, M, M - A))
            newA = np.where(pos_m, np.where(pos_a, M - A, M), np.where(pos_a, M + A, M))
            res[m], res[a] = newM.astype(np.float32), newA.astype(np.float32)
        w = window(n, self.bs0, bool(bf), prev_long, next_long)
        y = np.zeros((n, ch))
        for c in range(ch):
            if floors[c] is None:
                continue
            fl, d = floors[c]
            spec = fl.curve(d, n2).astype(np.float32) * res[c]
            y[:, c] = imdct(spec.astype(np.float32)) * w
        return y, n


def decode(data: bytes) -> Tuple[np.ndarray, int]:
    """Ogg/Vorbis bytes -> (float32 [frames, channels], sample rate)."""
    packets, last_gp = ogg_packets(data)
    dec = VorbisDecoder(packets)
    pcm = dec.decode()
    if last_gp >= 0 and pcm.shape[0] > last_gp:
        pcm = pcm[:last_gp]
    return pcm.astype(np.float32), dec.rate


def read_ogg(path: str) -> Tuple[np.ndarray, int]:
    with open(path, "rb") as f:
        return decode(f.read())
