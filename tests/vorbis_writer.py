"""Minimal Ogg/Vorbis ENCODER for tests (independent of genie_tts_amd/vorbis.py): writes
streams whose decoded output is known in closed form, from the Vorbis I specification's
bitstream description (Xiph.Org) and RFC 3533's Ogg framing.

The caller gives, per audio packet, the mode (short/long block), the window flags and per
channel a floor and a residue; the writer packs them.  Codebooks are complete trees (all
codeword lengths equal) or explicit length lists; VQ books use lookup type 1 or 2 with
values exactly representable in the Vorbis float format.  Floor 1 values are given as
the FINAL amplitude of each X point; the writer derives the coded differences with the
forward form of the spec's amplitude rule (prediction from the low/high neighbours).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np


class BitWriter:
    """LSb-first bit packing (Vorbis I section 2.1)."""

    def __init__(self):
        self.bits: List[int] = []

    def put(self, v: int, n: int):
        for i in range(n):
            self.bits.append((v >> i) & 1)

    def put_code(self, code: int, length: int):   # a Huffman codeword, MSb first
        for i in range(length - 1, -1, -1):
            self.bits.append((code >> i) & 1)

    def bytes(self) -> bytes:
        out = bytearray((len(self.bits) + 7) // 8)
        for i, b in enumerate(self.bits):
            out[i >> 3] |= b << (i & 7)
        return bytes(out)


def ilog(x: int) -> int:
    return 0 if x <= 0 else x.bit_length()


def float32_pack(v: float) -> int:
    """Vorbis float: v = mant * 2^(exp - 788), |mant| < 2^21 (exact for small dyadic values)."""
    if v == 0:
        return 0
    sign = 0x80000000 if v < 0 else 0
    m, e = abs(v), 0
    while m != int(m) or m >= (1 << 21):
        if m >= (1 << 21):
            m /= 2
            e += 1
        else:
            m *= 2
            e -= 1
    mant = int(m)
    return sign | ((e + 788) << 21) | mant


class Book:
    """A codebook: codeword lengths (0 = unused) and an optional VQ lookup."""

    def __init__(self, lengths: Sequence[int], dims: int = 1, lookup: int = 0, minimum: float = 0.0,
                 delta: float = 1.0, mults: Optional[Sequence[int]] = None, value_bits: int = 8,
                 seq: int = 0, ordered: bool = False):
        self.lengths = list(lengths)
        self.dims, self.lookup = dims, lookup
        self.minimum, self.delta, self.mults, self.value_bits, self.seq = minimum, delta, mults, value_bits, seq
        self.ordered = ordered
        self.codes = self._codes()

    def _codes(self):
        # canonical assignment in entry order: for equal lengths (the books built here) it is
        # simply entry index order within each length class -- checked against the
        # decoder's general rule by sorting on (length, entry) of a complete tree
        codes = {}
        used = [(i, l) for i, l in enumerate(self.lengths) if l > 0]
        if len(used) == 1:
            codes[used[0][0]] = (0, 1)
            return codes
        # a tree is filled left to right in entry order only when the lengths are
        # non-decreasing; the books here are built that way
        assert all(used[k][1] <= used[k + 1][1] for k in range(len(used) - 1)), "lengths must not decrease"
        code, prev = 0, used[0][1]
        for k, (i, l) in enumerate(used):
            if k:
                code = (code + 1) << (l - prev)
            prev = l
            codes[i] = (code, l)
        return codes

    def write_header(self, w: BitWriter):
        w.put(0x564342, 24)
        w.put(self.dims, 16)
        w.put(len(self.lengths), 24)
        if self.ordered:
            w.put(1, 1)
            cur = self.lengths[0]
            w.put(cur - 1, 5)
            i = 0
            n = len(self.lengths)
            while i < n:
                j = i
                while j < n and self.lengths[j] == cur:
                    j += 1
                w.put(j - i, ilog(n - i))
                i = j
                cur += 1
        else:
            w.put(0, 1)
            sparse = any(l == 0 for l in self.lengths)
            w.put(1 if sparse else 0, 1)
            for l in self.lengths:
                if sparse:
                    w.put(1 if l else 0, 1)
                    if l:
                        w.put(l - 1, 5)
                else:
                    w.put(l - 1, 5)
        w.put(self.lookup, 4)
        if self.lookup:
            w.put(float32_pack(self.minimum), 32)
            w.put(float32_pack(self.delta), 32)
            w.put(self.value_bits - 1, 4)
            w.put(self.seq, 1)
            for m in self.mults:
                w.put(m, self.value_bits)

    def write(self, w: BitWriter, entry: int):
        code, ln = self.codes[entry]
        w.put_code(code, ln)

    def vector(self, entry: int) -> np.ndarray:
        if self.lookup == 1:
            nval = len(self.mults)
            out, div, last = [], 1, 0.0
            for _ in range(self.dims):
                v = self.mults[(entry // div) % nval] * self.delta + self.minimum + last
                if self.seq:
                    last = v
                out.append(v)
                div *= nval
            return np.array(out)
        out, last = [], 0.0
        for d in range(self.dims):
            v = self.mults[entry * self.dims + d] * self.delta + self.minimum + last
            if self.seq:
                last = v
            out.append(v)
        return np.array(out)


def complete_book(entries: int, **kw) -> Book:
    return Book([int(math.log2(entries))] * entries, **kw)


# ---------------------------------------------------------------- floor 1
class Floor1Spec:
    def __init__(self, part_class, cdim, csub, cmaster, subbooks, mult, rangebits, xs):
        self.part_class, self.cdim, self.csub, self.cmaster = part_class, cdim, csub, cmaster
        self.subbooks, self.mult, self.rangebits, self.xs = subbooks, mult, rangebits, xs

    def write_header(self, w: BitWriter):
        w.put(1, 16)
        w.put(len(self.part_class), 5)
        for c in self.part_class:
            w.put(c, 4)
        for c in range(max(self.part_class) + 1 if self.part_class else 0):
            w.put(self.cdim[c] - 1, 3)
            w.put(self.csub[c], 2)
            if self.csub[c]:
                w.put(self.cmaster[c], 8)
            for b in self.subbooks[c]:
                w.put(b + 1, 8)
        w.put(self.mult - 1, 2)
        w.put(self.rangebits, 4)
        for x in self.xs[2:]:
            w.put(x, self.rangebits)

    RANGE = (256, 128, 86, 64)

    def predict(self, final: Sequence[int], i: int) -> int:
        """Point i's prediction: the line between its nearest earlier neighbours below and
        above in X, evaluated at X[i] (only final[:i] is read)."""
        xs = self.xs
        lo = max((j for j in range(i) if xs[j] < xs[i]), key=lambda j: xs[j])
        hi = min((j for j in range(i) if xs[j] > xs[i]), key=lambda j: xs[j])
        x0, y0, x1, y1 = xs[lo], final[lo], xs[hi], final[hi]
        dy, adx = y1 - y0, x1 - x0
        off = abs(dy) * (xs[i] - x0) // adx
        return y0 - off if dy < 0 else y0 + off

    def coded_values(self, final: Sequence[int]) -> List[int]:
        """The spec's amplitude rule run forward: final Y -> the values a packet carries."""
        rng = self.RANGE[self.mult - 1]
        out = [final[0], final[1]]
        for i in range(2, len(self.xs)):
            pred = self.predict(final, i)
            d = final[i] - pred
            highroom, lowroom = rng - pred, pred
            room = 2 * (highroom if highroom < lowroom else lowroom)
            if d == 0:
                out.append(0)
            elif d > 0 and 2 * d < room:
                out.append(2 * d)
            elif d < 0 and -2 * d - 1 < room:
                out.append(-2 * d - 1)
            elif highroom > lowroom:                # beyond the symmetric room: one-sided codes
                out.append(d + lowroom)
            else:
                out.append(highroom - 1 - d)
        return out

    def write_packet(self, w: BitWriter, final: Optional[Sequence[int]], books: List[Book]):
        if final is None:
            w.put(0, 1)
            return
        w.put(1, 1)
        rng = self.RANGE[self.mult - 1]
        vals = self.coded_values(final)
        w.put(vals[0], ilog(rng - 1))
        w.put(vals[1], ilog(rng - 1))
        off = 2
        for c in self.part_class:
            cdim, cbits = self.cdim[c], self.csub[c]
            # choose each value's subclass: the first subclass whose book can code it
            chosen = []
            for j in range(cdim):
                v = vals[off + j]
                sc = next(k for k in range(1 << cbits) if (self.subbooks[c][k] < 0 and v == 0) or
                          (self.subbooks[c][k] >= 0 and v < len(books[self.subbooks[c][k]].lengths)
                           and books[self.subbooks[c][k]].lengths[v] > 0))
                chosen.append(sc)
            if cbits:
                cval = 0
                for j in range(cdim - 1, -1, -1):
                    cval = (cval << cbits) | chosen[j]
                books[self.cmaster[c]].write(w, cval)
            for j in range(cdim):
                b = self.subbooks[c][chosen[j]]
                if b >= 0:
                    books[b].write(w, vals[off + j])
            off += cdim

    def curve(self, final: Sequence[int], n2: int) -> np.ndarray:
        """Expected floor: the lines between the used points (all points here), each
        y(x) = y0 + sign(dy) floor(|dy| (x - x0) / adx), extended flat to n2, through the
        dB table 10^((v - 255) 7 / 256)."""
        pts = sorted(zip(self.xs, [f * self.mult for f in final]))
        v = np.zeros(n2, np.int64)
        for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
            for x in range(x0, min(x1, n2)):
                dy = y1 - y0
                v[x] = y0 + (1 if dy >= 0 else -1) * (abs(dy) * (x - x0) // (x1 - x0))
        xl, yl = pts[-1]
        v[xl:] = yl
        return np.array([10.0 ** ((i - 255) * 7.0 / 256.0) for i in range(256)], np.float32)[v]


# ---------------------------------------------------------------- floor 0
class Floor0Spec:
    """Floor type 0 (LSP): header fields and packets; the expected curve is the spec's
    map/LSP formula evaluated here with numpy over the whole bark map (section 6.2.3)."""

    def __init__(self, order, rate, bark_size, amp_bits, amp_off, books):
        self.order, self.rate, self.bark_size = order, rate, bark_size
        self.amp_bits, self.amp_off, self.books = amp_bits, amp_off, books

    def write_header(self, w: BitWriter):
        w.put(0, 16)
        w.put(self.order, 8); w.put(self.rate, 16); w.put(self.bark_size, 16)
        w.put(self.amp_bits, 6); w.put(self.amp_off, 8)
        w.put(len(self.books) - 1, 4)
        for b in self.books:
            w.put(b, 8)

    def write_packet(self, w: BitWriter, dec, books: List[Book]):
        """dec = (amplitude, book index into self.books, VQ entries) or None (unused)."""
        if dec is None:
            w.put(0, self.amp_bits)
            return
        amp, bi, entries = dec
        w.put(amp, self.amp_bits)
        w.put(bi, ilog(len(self.books)))
        for e in entries:
            books[self.books[bi]].write(w, e)

    def coefficients(self, dec, books: List[Book]) -> np.ndarray:
        """Concatenated VQ vectors, each offset by the last scalar of the one before."""
        _, bi, entries = dec
        out, last = [], 0.0
        for e in entries:
            v = books[self.books[bi]].vector(e) + last
            out.extend(v.tolist())
            last = out[-1]
        return np.array(out[:self.order])

    def curve(self, dec, books: List[Book], n2: int) -> np.ndarray:
        amp = dec[0]
        c = np.cos(self.coefficients(dec, books))

        def bark(x):
            return 13.1 * np.arctan(0.00074 * x) + 2.24 * np.arctan(0.0000000185 * x * x) + 0.0001 * x
        i = np.arange(n2, dtype=np.float64)
        mp = np.minimum(self.bark_size - 1,
                        np.floor(bark(self.rate * i / (2.0 * n2)) * self.bark_size / bark(0.5 * self.rate)))
        cw = np.cos(np.pi * mp / self.bark_size)
        odd, even = c[1::2], c[0::2]
        po = np.prod(4.0 * (odd[None, :] - cw[:, None]) ** 2, axis=1)
        pe = np.prod(4.0 * (even[None, :] - cw[:, None]) ** 2, axis=1)
        if self.order % 2:
            p, q = (1.0 - cw * cw) * po, 0.25 * pe
        else:
            p, q = (1.0 - cw) / 2.0 * po, (1.0 + cw) / 2.0 * pe
        lin = np.exp(0.11512925 * (amp * self.amp_off / (((1 << self.amp_bits) - 1) * np.sqrt(p + q))
                                   - self.amp_off))
        return lin.astype(np.float32)


# ---------------------------------------------------------------- residue
class ResidueSpec:
    def __init__(self, rtype, begin, end, psize, nclass, classbook, books):
        self.rtype, self.begin, self.end, self.psize = rtype, begin, end, psize
        self.nclass, self.classbook, self.books = nclass, classbook, books   # books[class][pass]

    def write_header(self, w: BitWriter):
        w.put(self.rtype, 16)
        w.put(self.begin, 24)
        w.put(self.end, 24)
        w.put(self.psize - 1, 24)
        w.put(self.nclass - 1, 6)
        w.put(self.classbook, 8)
        for bk in self.books:
            casc = sum(1 << j for j in range(8) if bk[j] >= 0)
            w.put(casc & 7, 3)
            if casc >> 3:
                w.put(1, 1)
                w.put(casc >> 3, 5)
            else:
                w.put(0, 1)
        for bk in self.books:
            for j in range(8):
                if bk[j] >= 0:
                    w.put(bk[j], 8)

    def write_packet(self, w: BitWriter, vecs: List[np.ndarray], classes: List[List[int]],
                     entries: List[List[List[List[int]]]], books: List[Book], n2: int, skip: List[bool]):
        """classes[ch][partition]; entries[ch][partition][pass] = VQ entries of that pass.
        For type 2, one interleaved vector (ch = 1 here)."""
        cb = books[self.classbook]
        size = n2 * (len(skip) if self.rtype == 2 else 1)
        nparts = (min(self.end, size) - min(self.begin, size)) // self.psize
        cpw = cb.dims
        nvec = 1 if self.rtype == 2 else len(skip)
        sk = [all(skip)] if self.rtype == 2 else skip
        for pss in range(8):
            pc = 0
            while pc < nparts:
                if pss == 0:
                    for j in range(nvec):
                        if sk[j]:
                            continue
                        code = 0
                        for i in range(cpw):
                            c = classes[j][pc + i] if pc + i < nparts else 0
                            code = code * self.nclass + c
                        cb.write(w, code)
                for _ in range(cpw):
                    if pc >= nparts:
                        break
                    for j in range(nvec):
                        if sk[j]:
                            continue
                        bk = self.books[classes[j][pc]][pss]
                        if bk >= 0:
                            for e in entries[j][pc][pss]:
                                books[bk].write(w, e)
                    pc += 1


# ---------------------------------------------------------------- stream
def ogg_crc(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b << 24
        for _ in range(8):
            c = ((c << 1) ^ 0x04C11DB7) & 0xFFFFFFFF if c & 0x80000000 else (c << 1) & 0xFFFFFFFF
    return c


def ogg_page(packets_data: List[bytes], granule: int, seq: int, serial: int, bos=False, eos=False,
             continued=False) -> bytes:
    lace = []
    body = b""
    for p in packets_data:
        n = len(p)
        while n >= 255:
            lace.append(255)
            n -= 255
        lace.append(n)
        body += p
    hdr = bytearray(b"OggS") + bytes([0, (1 if continued else 0) | (2 if bos else 0) | (4 if eos else 0)])
    hdr += granule.to_bytes(8, "little", signed=True) + serial.to_bytes(4, "little") + seq.to_bytes(4, "little")
    hdr += b"\0\0\0\0" + bytes([len(lace)]) + bytes(lace)
    page = bytearray(hdr + body)
    page[22:26] = ogg_crc(bytes(page)).to_bytes(4, "little")
    return bytes(page)


def ident_packet(channels: int, rate: int, bs0: int, bs1: int) -> bytes:
    w = BitWriter()
    w.put(1, 8)
    for ch in b"vorbis":
        w.put(ch, 8)
    w.put(0, 32); w.put(channels, 8); w.put(rate, 32)
    w.put(0, 32); w.put(128000, 32); w.put(0, 32)
    w.put(int(math.log2(bs0)), 4); w.put(int(math.log2(bs1)), 4); w.put(1, 1)
    return w.bytes()


def comment_packet() -> bytes:
    w = BitWriter()
    w.put(3, 8)
    for ch in b"vorbis":
        w.put(ch, 8)
    vendor = b"genie test writer"
    w.put(len(vendor), 32)
    for ch in vendor:
        w.put(ch, 8)
    w.put(0, 32)
    w.put(1, 1)
    return w.bytes()


def setup_packet(books: List[Book], floors: List, residues: List[ResidueSpec], mappings, modes,
                 channels: int) -> bytes:
    w = BitWriter()
    w.put(5, 8)
    for ch in b"vorbis":
        w.put(ch, 8)
    w.put(len(books) - 1, 8)
    for b in books:
        b.write_header(w)
    w.put(0, 6); w.put(0, 16)                       # one time-domain placeholder
    w.put(len(floors) - 1, 6)
    for f in floors:
        f.write_header(w)
    w.put(len(residues) - 1, 6)
    for r in residues:
        r.write_header(w)
    w.put(len(mappings) - 1, 6)
    for coupling, floor, residue in mappings:
        w.put(0, 16)
        w.put(0, 1)                                 # one submap
        if coupling:
            w.put(1, 1)
            w.put(len(coupling) - 1, 8)
            for m, a in coupling:
                w.put(m, ilog(channels - 1)); w.put(a, ilog(channels - 1))
        else:
            w.put(0, 1)
        w.put(0, 2)
        w.put(0, 8); w.put(floor, 8); w.put(residue, 8)
    w.put(len(modes) - 1, 6)
    for bf, mapping in modes:
        w.put(bf, 1); w.put(0, 16); w.put(0, 16); w.put(mapping, 8)
    w.put(1, 1)
    return w.bytes()


def stream(headers: List[bytes], audio: List[bytes], samples_per_packet: List[int], serial: int = 0x5EED,
           per_page: int = 3, total: Optional[int] = None) -> bytes:
    out = ogg_page([headers[0]], 0, 0, serial, bos=True)
    out += ogg_page(headers[1:], 0, 1, serial)
    seq, gp = 2, 0
    for i in range(0, len(audio), per_page):
        chunk = audio[i:i + per_page]
        gp += sum(samples_per_packet[i:i + per_page])
        last = i + per_page >= len(audio)
        g = total if (last and total is not None) else gp
        out += ogg_page(chunk, g, seq, serial, eos=last)
        seq += 1
    return out
