"""CPU: the Ogg/Vorbis reader for reference clips (genie_tts_amd/vorbis.py; the reference
reads '.ogg' through libsndfile, Audio/Audio.py:24, Internal.py:38) against streams built by
an independent test encoder (tests/vorbis_writer.py) whose decoded output is computed here
in closed form: floor-1 lines y0 + sign(dy) floor(|dy| dx / adx) through the dB table,
residue vectors summed from the chosen VQ entries, the spec's inverse coupling, a direct
O(N^2) cosine-sum IMDCT, the spec's window slopes and overlap-add on an absolute timeline.

libvorbis itself is not in this image, so the absolute output scale rests on the
specification's (and libvorbis') unnormalised inverse MDCT: parity against libvorbis'
PCM is unpinned; every decoding step above is pinned by these round trips."""
import math

import numpy as np
import pytest

from genie_tts_amd import audio as A
from genie_tts_amd import vorbis
from tests import vorbis_writer as W

BS0, BS1 = 256, 2048


def _books(seed=0):
    r = np.random.default_rng(seed)
    return [
        W.complete_book(256),                                         # 0: floor Y values
        W.complete_book(8),                                           # 1: floor class-1 master
        W.Book([2, 0, 3, 3, 0, 3, 3, 3, 3]),                          # 2: sparse (1, 4 unused)
        W.complete_book(4, dims=2),                                   # 3: residue classbook
        W.complete_book(256, dims=2, lookup=1, minimum=-7.5, delta=1.0,
                        mults=list(range(16)), value_bits=4),         # 4: lookup 1
        W.Book([2, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5, 6, 6], dims=4, lookup=2,
               minimum=-8.0, delta=0.5, mults=r.integers(0, 16, 64).tolist(), value_bits=4,
               seq=1, ordered=True),                                  # 5: lookup 2, sequence
        W.complete_book(16, dims=2, lookup=1, minimum=0.375, delta=0.046875,
                        mults=[0, 1, 2, 3], value_bits=2, seq=1),     # 6: floor-0 LSP steps
    ]


def _floors():
    kw = dict(part_class=[0, 1, 0], cdim=[2, 3], csub=[0, 1], cmaster=[-1, 1], subbooks=[[2], [-1, 0]], mult=2)
    return [W.Floor1Spec(rangebits=7, xs=[0, 128, 64, 32, 96, 16, 48, 80, 112], **kw),
            W.Floor1Spec(rangebits=10, xs=[0, 1024, 512, 128, 768, 32, 256, 640, 900], **kw)]


RBOOKS = [[4, -1, 5, -1, -1, -1, -1, -1], [-1, 4, -1, 5, -1, -1, -1, -1]]   # [class][pass]


def _residues(rtype):
    k = 2 if rtype == 2 else 1
    return [W.ResidueSpec(rtype, 0, 128 * k, 16, 2, 3, RBOOKS),
            W.ResidueSpec(rtype, 0, (1024 - 64) * k, 16, 2, 3, RBOOKS)]


def _finals(fl: W.Floor1Spec, r) -> list:
    """Final amplitudes with every coded value nonzero (all points drawn): class-0 points
    (the sparse book) use small steps whose codes the book holds, class-1 points jump
    anywhere, including beyond the symmetric room (one-sided codes)."""
    final = [int(r.integers(10, 118)), int(r.integers(10, 118))]
    kinds = [c for c in fl.part_class for _ in range(fl.cdim[c])]
    for i in range(2, len(fl.xs)):
        pred = fl.predict(final, i)
        if kinds[i - 2] == 0:
            ok = [d for d in (1, -2, -3, 3, -4, 4) if 0 <= pred + d < 128]
            final.append(pred + int(r.choice(ok)))
        else:
            v = int(r.integers(0, 128))
            final.append(v if v != pred else (v + 1) % 128)
    vals = fl.coded_values(final)
    assert all(v != 0 for v in vals[2:])
    return final


def _couple_inverse(M, A_):
    """The spec's square-polar inverse coupling, element by element."""
    m, a = M.copy(), A_.copy()
    for i in range(M.shape[0]):
        mm, aa = float(M[i]), float(A_[i])
        if mm > 0:
            m[i], a[i] = (mm, mm - aa) if aa > 0 else (mm + aa, mm)
        else:
            m[i], a[i] = (mm, mm + aa) if aa > 0 else (mm - aa, mm)
    return m, a


def _imdct_direct(X):
    n = 2 * len(X)
    i = np.arange(n)[:, None]
    k = np.arange(len(X))[None, :]
    return np.cos(np.pi / (2 * n) * (2 * i + 1 + n / 2) * (2 * k + 1)) @ np.asarray(X, np.float64)


def _slope(i, start, ln, rising):
    x = (i - start + 0.5) / ln * math.pi / 2 + (0 if rising else math.pi / 2)
    return math.sin(math.pi / 2 * math.sin(x) ** 2)


def _window(n, long_block, prev_long, next_long):
    w = np.zeros(n)
    if long_block and not prev_long:
        ls, ln = n // 4 - BS0 // 4, BS0 // 2
    else:
        ls, ln = 0, n // 2
    if long_block and not next_long:
        rs, rn = 3 * n // 4 - BS0 // 4, BS0 // 2
    else:
        rs, rn = n // 2, n // 2
    for i in range(n):
        if i < ls:
            w[i] = 0.0
        elif i < ls + ln:
            w[i] = _slope(i, ls, ln, True)
        elif i < rs:
            w[i] = 1.0
        elif i < rs + rn:
            w[i] = _slope(i, rs, rn, False)
    return w


def _packet(books, floors, residues, rtype, mode, prev_long, next_long, used, r):
    """One audio packet and its expected windowed time-domain frame [n, 2]."""
    n = BS1 if mode else BS0
    n2 = n // 2
    w = W.BitWriter()
    w.put(0, 1)
    w.put(mode, 1)
    if mode:
        w.put(int(prev_long), 1)
        w.put(int(next_long), 1)
    fl = floors[mode]
    if isinstance(fl, W.Floor0Spec):
        # amplitude and LSP entries; the coefficients ascend through (0, pi) like real line
        # spectral pairs (book 6 steps 0.375..0.52, each vector offset by the previous one's last)
        nvq = -(-fl.order // books[fl.books[0]].dims)
        finals = [(int(r.integers(1, 1 << fl.amp_bits)), 0, [int(r.integers(0, 16)) for _ in range(nvq)])
                  if used[c] else None for c in range(2)]
    else:
        finals = [_finals(fl, r) if used[c] else None for c in range(2)]
    for c in range(2):
        fl.write_packet(w, finals[c], books)
    nonzero = any(used)                                 # channels 0 and 1 are coupled
    skip = [not nonzero] * 2
    res = residues[mode]
    size = n2 * 2 if rtype == 2 else n2
    nparts = min(res.end, size) // res.psize
    nvec = 1 if rtype == 2 else 2
    classes = [[int(r.integers(0, 2)) for _ in range(nparts)] for _ in range(nvec)]
    entries = [[[[] for _ in range(8)] for _ in range(nparts)] for _ in range(nvec)]
    vecs = [np.zeros(size) for _ in range(nvec)]
    for j in range(nvec):
        for p in range(nparts):
            for pss in range(8):
                bk = RBOOKS[classes[j][p]][pss]
                if bk < 0:
                    continue
                book = books[bk]
                es = [int(r.integers(0, len(book.lengths))) for _ in range(res.psize // book.dims)]
                entries[j][p][pss] = es
                off = p * res.psize
                step = res.psize // book.dims
                for i, e in enumerate(es):
                    v = book.vector(e)
                    for d in range(book.dims):
                        at = off + i + d * step if rtype == 0 else off + i * book.dims + d
                        vecs[j][at] += v[d]
    res.write_packet(w, vecs, classes, entries, books, n2, skip)
    if not nonzero:
        rv = [np.zeros(n2), np.zeros(n2)]
    elif rtype == 2:
        rv = [vecs[0][0::2], vecs[0][1::2]]
    else:
        rv = vecs
    rv = [x.astype(np.float32) for x in rv]
    m, a = _couple_inverse(rv[0], rv[1])
    win = _window(n, bool(mode), prev_long, next_long)
    y = np.zeros((n, 2))
    for c, spec in enumerate((m, a)):
        if finals[c] is not None:
            curve = fl.curve(finals[c], books, n2) if isinstance(fl, W.Floor0Spec) else fl.curve(finals[c], n2)
            y[:, c] = _imdct_direct(curve.astype(np.float64) * spec) * win
    return w.bytes(), y


def _floors0():
    """Floor type 0 for both block sizes: LSP orders 6 (even) and 5 (odd), different bark maps."""
    return [W.Floor0Spec(order=6, rate=32000, bark_size=64, amp_bits=6, amp_off=3, books=[6]),
            W.Floor0Spec(order=5, rate=32000, bark_size=256, amp_bits=8, amp_off=3, books=[6, 6])]


def _build(rtype, modes, used=None, seed=0, total_trim=0, floors=None):
    r = np.random.default_rng(seed)
    books, floors, residues = _books(seed), floors or _floors(), _residues(rtype)
    mappings = [([(0, 1)], 0, 0), ([(0, 1)], 1, 1)]
    headers = [W.ident_packet(2, 32000, BS0, BS1), W.comment_packet(),
               W.setup_packet(books, floors, residues, mappings, [(0, 0), (1, 1)], 2)]
    used = used or [(True, True)] * len(modes)
    pkts, frames, ns = [], [], []
    for k, mode in enumerate(modes):
        prev_long = k > 0 and modes[k - 1] == 1
        next_long = k + 1 < len(modes) and modes[k + 1] == 1
        b, y = _packet(books, floors, residues, rtype, mode, prev_long, next_long, used[k], r)
        pkts.append(b)
        frames.append(y)
        ns.append(BS1 if mode else BS0)
    # absolute timeline: frame k starts where its left overlap centre meets frame k-1's right one
    starts = [0]
    for k in range(1, len(ns)):
        starts.append(starts[-1] + 3 * ns[k - 1] // 4 - ns[k] // 4)
    lo = min(starts)                                    # a long frame after a short one starts earlier
    starts = [s - lo for s in starts]
    buf = np.zeros((max(s + n for s, n in zip(starts, ns)), 2))
    for s, y in zip(starts, frames):
        buf[s:s + y.shape[0]] += y
    expect = buf[starts[0] + ns[0] // 2: starts[-1] + ns[-1] // 2]
    per = [0] + [ns[k - 1] // 4 + ns[k] // 4 for k in range(1, len(ns))]
    total = sum(per) - total_trim
    data = W.stream(headers, pkts, per, total=total)
    return data, expect[:total]


MODES = [1, 1, 0, 0, 1, 0, 1, 1, 0]        # long/short transitions both ways


@pytest.mark.parametrize("rtype", [0, 1, 2])
def test_round_trip_residue_types_long_short(rtype):
    data, expect = _build(rtype, MODES, seed=rtype)
    pcm, rate = vorbis.decode(data)
    assert rate == 32000 and pcm.shape == expect.shape and pcm.dtype == np.float32
    scale = np.abs(expect).max()
    assert scale > 1.0
    np.testing.assert_allclose(pcm, expect, rtol=0, atol=2e-6 * scale)


@pytest.mark.parametrize("rtype", [1, 2])
def test_round_trip_floor0(rtype):
    """Floor type 0 (LSP curve over the bark map, Vorbis I section 6) for both block sizes,
    even and odd order, with one silent channel per packet in places: the decoder's curve,
    times the residue, through the IMDCT and overlap-add, equals the closed form."""
    used = [(True, True), (True, False), (True, True), (False, True), (True, True), (True, True)]
    data, expect = _build(rtype, [1, 0, 0, 1, 1, 0], used=used, seed=20 + rtype, floors=_floors0())
    pcm, rate = vorbis.decode(data)
    assert rate == 32000 and pcm.shape == expect.shape
    assert np.isfinite(expect).all()
    scale = np.abs(expect).max()
    assert scale > 0.1
    np.testing.assert_allclose(pcm, expect, rtol=0, atol=2e-6 * scale)


def test_floor0_curve_matches_the_spec_formula():
    """The decoder's floor-0 curve alone (its run-length loop over equal map values) against
    the vectorised spec formula, for both orders and several amplitudes."""
    books = _books(0)
    r = np.random.default_rng(7)
    for spec in _floors0():
        bits = W.BitWriter()
        spec.write_header(bits)
        dec_fl = vorbis.Floor0(_bits_after_type(bits))
        for _ in range(4):
            nvq = -(-spec.order // 2)
            dec = (int(r.integers(1, 1 << spec.amp_bits)), 0, [int(r.integers(0, 16)) for _ in range(nvq)])
            coef = spec.coefficients(dec, books).tolist()
            for n2 in (128, 1024):
                got = dec_fl.curve((dec[0], coef), n2)
                np.testing.assert_allclose(got, spec.curve(dec, books, n2), rtol=2e-6)


def _bits_after_type(bits: "W.BitWriter"):
    """A reader positioned after the 16-bit floor type of a written floor header."""
    r = vorbis._Bits(bits.bytes())
    assert r.read(16) == 0
    return r


def test_unused_floors_and_granule_trim():
    """A channel whose floor is unused is silent but its residue still takes part in the
    coupling; both unused: no residue is coded; the last page's granule trims the end."""
    used = [(True, True), (True, False), (False, True), (False, False), (True, True)]
    data, expect = _build(1, [1, 0, 0, 1, 1], used=used, seed=5, total_trim=100)
    pcm, _ = vorbis.decode(data)
    assert pcm.shape == expect.shape
    np.testing.assert_allclose(pcm, expect, rtol=0, atol=2e-6 * np.abs(expect).max())


def test_fast_imdct_equals_cosine_sum():
    r = np.random.default_rng(1)
    for m in (32, 128, 1024):
        X = r.normal(size=m)
        np.testing.assert_allclose(vorbis.imdct(X), _imdct_direct(X), atol=1e-9 * m)


@pytest.mark.parametrize("prev_long,next_long", [(False, False), (False, True), (True, False), (True, True)])
def test_window_matches_spec_and_is_power_complementary(prev_long, next_long):
    w = vorbis.window(BS1, BS0, True, prev_long, next_long)
    np.testing.assert_allclose(w, _window(BS1, True, prev_long, next_long), atol=1e-12)
    s = vorbis.window(BS0, BS0, False, True, True)
    # the short window's halves overlap one another: w(i)^2 + w(i + n/2)^2 = 1
    np.testing.assert_allclose(s[:BS0 // 2] ** 2 + s[BS0 // 2:] ** 2, 1.0, atol=1e-12)


def test_codebook_codeword_assignment():
    """Entry-order assignment of the lowest free codeword per length: an unordered tree
    whose lengths go up and down, decoded entry by entry from its canonical codes."""
    lengths = [2, 3, 3, 2, 3, 3]                        # 1/4 + 1/8 + 1/8 + 1/4 + 1/8 + 1/8 = 1
    codes = vorbis.Codebook._assign(lengths)
    # entry 0 -> 00, 1 -> 010, 2 -> 011, 3 -> 10, 4 -> 110, 5 -> 111
    assert codes == {(2, 0b00): 0, (3, 0b010): 1, (3, 0b011): 2, (2, 0b10): 3, (3, 0b110): 4, (3, 0b111): 5}


def test_crc_mismatch_and_missing_headers_are_errors():
    data, _ = _build(1, [1, 1], seed=3)
    bad = bytearray(data)
    bad[-3] ^= 0x40
    with pytest.raises(vorbis.VorbisError):
        vorbis.decode(bytes(bad))
    with pytest.raises(vorbis.VorbisError):
        vorbis.decode(data[:data.index(b"OggS", 4)])    # the identification page only


def test_load_audio_ogg_equals_float_wav(tmp_path):
    """load_audio on '.ogg' = the same decoded samples as an IEEE-float .wav (mono mix,
    resample to 32 kHz, +0.3 s; Audio.py:19-51)."""
    data, _ = _build(2, [1] * 20 + [0, 0, 1] * 4, seed=11)
    raw, rate = vorbis.decode(data)
    og = tmp_path / "ref.ogg"
    og.write_bytes(data)
    wv = tmp_path / "ref.wav"
    _write_float_wav(wv, raw, rate)
    assert ".ogg" in A.SUPPORTED_AUDIO_EXTS
    a, b = A.load_audio(str(og), 32000), A.load_audio(str(wv), 32000)
    np.testing.assert_array_equal(a, b)


def _write_float_wav(path, x, rate):
    ch = x.shape[1]
    body = x.astype("<f4").tobytes()
    fmt = (3).to_bytes(2, "little") + ch.to_bytes(2, "little") + rate.to_bytes(4, "little") + \
        (rate * 4 * ch).to_bytes(4, "little") + (4 * ch).to_bytes(2, "little") + (32).to_bytes(2, "little")
    riff = b"WAVE" + b"fmt " + len(fmt).to_bytes(4, "little") + fmt + b"data" + len(body).to_bytes(4, "little") + body
    path.write_bytes(b"RIFF" + len(riff).to_bytes(4, "little") + riff)
