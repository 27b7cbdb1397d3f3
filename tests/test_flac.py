"""CPU: the FLAC reader for reference clips (genie_tts_amd/flac.py; the reference reads
.flac through libsndfile, Audio/Audio.py:24, Internal.py:38) against an independent
test encoder (tests/flac_writer.py): lossless round trips over every subframe type,
residual coding, channel assignment and header form, CRC checks, and load_audio on a
.flac equal to the same samples as a .wav."""
import wave

import numpy as np
import pytest

from genie_tts_amd import audio as A
from genie_tts_amd import flac
from tests.flac_writer import encode


def _sig(n, ch, bps, seed=0):
    r = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) * 0.6
    x = np.stack([amp * np.sin(2 * np.pi * (0.01 + 0.003 * c) * t) + r.normal(0, amp * 0.01, n) for c in range(ch)], 1)
    return np.clip(np.round(x), -(1 << (bps - 1)), (1 << (bps - 1)) - 1).astype(np.int64)


LPC = dict(kind="lpc", coef=[1843, -870], shift=10, prec=12)


@pytest.mark.parametrize("sub", [
    dict(kind="verbatim"),
    dict(kind="fixed", order=0), dict(kind="fixed", order=1), dict(kind="fixed", order=2, porder=2),
    dict(kind="fixed", order=3, rice2=True), dict(kind="fixed", order=4, porder=3, escape=True),
    dict(LPC), dict(LPC, porder=2, rice2=True, escape=True),
    dict(kind="lpc", coef=[700, 500, -300, 100, 20, -5, 3, 1], shift=11, prec=13, porder=1),
])
def test_mono_subframe_types_round_trip(sub):
    x = _sig(1024 + 576, 1, 16)
    data = encode(x, 32000, 16, [dict(n=1024, mode=0, sub=[sub]), dict(n=576, mode=0, sub=[sub])])
    pcm, rate, bps = flac.decode(data)
    assert rate == 32000 and bps == 16 and np.array_equal(pcm, x)


@pytest.mark.parametrize("mode", [1, 8, 9, 10])   # independent, left/side, side/right, mid/side
def test_stereo_channel_assignments(mode):
    x = _sig(4096, 2, 16, seed=mode)
    sub = [dict(kind="fixed", order=2, porder=4), dict(LPC, porder=1)]
    data = encode(x, 44100, 16, [dict(n=4096, mode=mode, sub=sub)], header_rate=True)
    pcm, rate, _ = flac.decode(data)
    assert rate == 44100 and np.array_equal(pcm, x)


def test_constant_wasted_bits_24bit_variable_blocks_odd_rate():
    x = _sig(300 + 200 + 1000, 1, 24) & ~0xFF           # low 8 bits zero: wasted bits
    x[300:500] = 4096
    frames = [dict(n=300, mode=0, sub=[dict(kind="fixed", order=2, wasted=8)]),
              dict(n=200, mode=0, sub=[dict(kind="constant")]),
              dict(n=1000, mode=0, sub=[dict(LPC, wasted=3, porder=3)])]
    data = encode(x, 22222, 24, frames, variable=True, header_rate=True, header_size=False)
    pcm, rate, bps = flac.decode(data)
    assert rate == 22222 and bps == 24 and np.array_equal(pcm, x)


def test_crc_mismatch_is_an_error():
    x = _sig(1024, 1, 16)
    data = bytearray(encode(x, 32000, 16, [dict(n=1024, mode=0, sub=[dict(kind="fixed", order=2)])]))
    data[-5] ^= 0x10
    with pytest.raises(flac.FlacError):
        flac.decode(bytes(data))


def test_load_audio_flac_equals_wav(tmp_path):
    """The same 16-bit stereo clip as .flac and .wav: identical 32 kHz mono + 0.3 s
    (Audio.py:19-51; libsndfile scales 16-bit PCM by 1/32768 for both)."""
    x = _sig(3 * 24000, 2, 16, seed=7)
    fl = tmp_path / "ref.flac"
    fl.write_bytes(encode(x, 24000, 16, [dict(n=4608, mode=10, sub=[dict(LPC, porder=2), dict(kind="fixed", order=1)])
                                         for _ in range(15)] + [dict(n=3 * 24000 - 15 * 4608, mode=1,
                                                                     sub=[dict(kind="verbatim")] * 2)]))
    wv = tmp_path / "ref.wav"
    with wave.open(str(wv), "wb") as wf:
        wf.setnchannels(2); wf.setsampwidth(2); wf.setframerate(24000)
        wf.writeframes(x.astype("<i2").tobytes())
    assert ".flac" in A.SUPPORTED_AUDIO_EXTS
    a, b = A.load_audio(str(fl), 32000), A.load_audio(str(wv), 32000)
    assert a.shape == b.shape == (int(np.ceil(3 * 32000)) + int(0.3 * 32000),)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("tail", [b"TAG" + bytes(125), bytes(64), b"\xff\xf8junk\xff\xf9\x00\x00"])
def test_trailing_bytes_after_the_last_frame(tail):
    """an ID3v1 'TAG' block, zero padding or junk holding a sync pattern after
    the last frame is not audio (libsndfile reads such files): decoding stops at
    STREAMINFO's sample count, or resynchronises and finds no further frame."""
    x = _sig(1024 + 576, 1, 16)
    frames = [dict(n=1024, mode=0, sub=[dict(LPC)]), dict(n=576, mode=0, sub=[dict(kind="fixed", order=2)])]
    data = encode(x, 32000, 16, frames)
    pcm, _, _ = flac.decode(data + tail)
    assert np.array_equal(pcm, x)
    # STREAMINFO total 0 (unknown): the same bytes end at the last real frame too
    i = data.index(b"fLaC") + 4 + 4 + 13             # STREAMINFO body byte 13: total samples start
    body = bytearray(data)
    body[i] &= 0xF0
    body[i + 1:i + 5] = bytes(4)
    pcm, _, _ = flac.decode(bytes(body) + tail)
    assert np.array_equal(pcm, x)
