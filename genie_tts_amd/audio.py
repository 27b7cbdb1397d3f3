"""Reference-audio loading for `set_reference_audio`, following
src/genie_tts/Audio/Audio.py:19-51 and Audio/ReferenceAudio.py:28-57:

  read -> float32 -> mono (mean over channels) -> resample to the target rate
  -> warn outside 3..10 s -> append 0.3 s of silence;
  audio_32k = load(path, 32000); audio_16k = resample(audio_32k, 32000 -> 16000).

The reference reads with libsndfile (soundfile) and resamples with soxr 'hq';
neither exists in this image, so reading is our own RIFF/WAVE (PCM 8/16/24/32,
IEEE float 32/64), AIFF, FLAC (flac.py, lossless: exact samples) and Ogg/Vorbis
(vorbis.py, the Vorbis I float decode; Ogg parity with libsndfile/libvorbis is
UNPINNED: only round trips through the repo's own test encoder check it, no
libvorbis-encoded clip exists here) parsers, and
resampling is a rational polyphase Kaiser-windowed sinc
(scipy.signal.resample_poly), NOT soxr's HQ filter.  Host-side, once per
reference clip.  Parity with soxr is unpinned (a different filter: any clip not
already at 32 kHz / the 32 -> 16 kHz step differ at the filter level);
equal-length outputs are guaranteed (ceil(n * out / in) like soxr).
"""
from __future__ import annotations

import logging
import math
import os
import struct
from typing import Optional, Tuple

import numpy as np

logger = logging.getLogger(__name__)

MIN_DURATION_S = 3
MAX_DURATION_S = 10
SILENCE_TO_APPEND_S = 0.3
SUPPORTED_AUDIO_EXTS = {".wav", ".flac", ".ogg", ".aiff", ".aif"}   # Internal.py:38 (+ AIFF)


def _pcm_to_float(raw: bytes, width: int, big_endian: bool = False) -> np.ndarray:
    if width == 1:                                           # WAV 8-bit is unsigned
        return (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    if width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = (b[:, 0] << 16 | b[:, 1] << 8 | b[:, 2]) if big_endian else (b[:, 2] << 16 | b[:, 1] << 8 | b[:, 0])
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        return v.astype(np.float32) / float(1 << 23)
    dt = {2: "i2", 4: "i4"}[width]
    v = np.frombuffer(raw, (">" if big_endian else "<") + dt)
    return v.astype(np.float32) / float(1 << (8 * width - 1))


def read_wav(path: str) -> Tuple[np.ndarray, int]:
    """-> (float32 [frames, channels], sample rate) for RIFF/WAVE files."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:              # WAVE_FORMAT_EXTENSIBLE: sub-format GUID
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, bits = fmt
    if tag == 1:
        x = _pcm_to_float(pcm[:len(pcm) - len(pcm) % (ch * bits // 8)], bits // 8)
    elif tag == 3 and bits in (32, 64):
        x = np.frombuffer(pcm[:len(pcm) - len(pcm) % (ch * bits // 8)], "<f4" if bits == 32 else "<f8")
        x = x.astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAV format tag {tag} / {bits} bits")
    return x.reshape(-1, ch), sr


def read_aiff(path: str) -> Tuple[np.ndarray, int]:
    import aifc   # stdlib (deprecated in 3.11+, present in 3.10)
    with aifc.open(path, "rb") as a:
        ch, width, sr, n = a.getnchannels(), a.getsampwidth(), a.getframerate(), a.getnframes()
        raw = a.readframes(n)
    return _pcm_to_float(raw, width, big_endian=True).reshape(-1, ch), sr


def read_audio(path: str) -> Tuple[np.ndarray, int]:
    ext = os.path.splitext(path)[1].lower()
    if ext == ".wav":
        return read_wav(path)
    if ext in (".aiff", ".aif"):
        return read_aiff(path)
    if ext == ".flac":
        from .flac import read_flac
        return read_flac(path)
    if ext == ".ogg":
        from .vorbis import read_ogg
        return read_ogg(path)
    raise ValueError(f"audio format '{ext}' is not supported (supported: {sorted(SUPPORTED_AUDIO_EXTS)})")


def resample(x: np.ndarray, sr_in: int, sr_out: int) -> np.ndarray:
    """1-D float32 resampling sr_in -> sr_out, output length ceil(n * sr_out / sr_in)."""
    x = np.asarray(x, np.float32)
    if sr_in == sr_out:
        return x.copy()
    from scipy.signal import resample_poly
    g = math.gcd(int(sr_in), int(sr_out))
    up, down = int(sr_out) // g, int(sr_in) // g
    y = resample_poly(x.astype(np.float64), up, down)
    n = -(-x.shape[0] * up // down)
    return y[:n].astype(np.float32)


def load_audio(path: str, target_sampling_rate: int = 32000) -> np.ndarray:
    """Audio.py:19-51: float32 mono at the target rate + 0.3 s of silence (1-D)."""
    wav, sr = read_audio(os.fspath(path))
    wav = wav.mean(axis=1) if wav.shape[1] > 1 else wav[:, 0]
    wav = resample(wav, sr, target_sampling_rate)
    lo, hi = int(MIN_DURATION_S * target_sampling_rate), int(MAX_DURATION_S * target_sampling_rate)
    if not lo <= wav.shape[0] <= hi:
        logger.warning("The reference audio '%s' has a duration of %.2f seconds, which is outside the "
                       "recommended range of %d to %d seconds!", os.path.basename(path),
                       wav.shape[0] / target_sampling_rate, MIN_DURATION_S, MAX_DURATION_S)
    silence = np.zeros(int(SILENCE_TO_APPEND_S * target_sampling_rate), np.float32)
    return np.concatenate([wav, silence]).astype(np.float32)


def write_wav(path: str, audio: np.ndarray, sample_rate: int = 32000) -> None:
    """16-bit mono WAV as the reference's TTSPlayer writes it (x * 32767 -> int16)."""
    import wave
    parent = os.path.dirname(path)
    if parent:
        os.makedirs(parent, exist_ok=True)
    with wave.open(path, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sample_rate)
        wf.writeframes(to_pcm16(audio))


def to_pcm16(audio: np.ndarray) -> bytes:
    """TTSPlayer._preprocess_for_playback: (x * 32767).astype(int16) bytes."""
    return (np.asarray(audio, np.float32).squeeze() * 32767).astype(np.int16).tobytes()
