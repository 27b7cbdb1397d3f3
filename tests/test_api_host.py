"""CPU: the drop-in API's host side -- TextSplitter against the reference's own
outputs (tests/golden/text_splitter.json, tests/golden/make_text_splitter.py),
reference-clip loading (Audio.py:19-51: mono, resample, 0.3 s silence; soxr is
absent, so the resampler is checked on lengths and a band-limited tone, parity
with soxr unpinned), and set_reference_audio's bookkeeping."""
import json
import os
import wave

import numpy as np
import pytest

from genie_tts_amd import audio as A
from genie_tts_amd.text_splitter import TextSplitter

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_text_splitter_matches_reference_outputs():
    cases = json.load(open(os.path.join(GOLD, "text_splitter.json"), encoding="utf-8"))
    assert len(cases) >= 30
    for c in cases:
        assert TextSplitter(c["max_len"], c["min_len"]).split(c["text"]) == c["split"], c["text"]


def _write(path, x, sr, width=2, channels=1):
    x = np.asarray(x, np.float64).reshape(-1, channels)
    with wave.open(path, "wb") as wf:
        wf.setnchannels(channels)
        wf.setsampwidth(width)
        wf.setframerate(sr)
        scale = float(1 << (8 * width - 1)) - 1
        dt = {2: "<i2", 4: "<i4"}[width]
        wf.writeframes(np.round(x * scale).astype(dt).tobytes())


@pytest.mark.parametrize("sr,width,ch", [(48000, 2, 1), (44100, 2, 2), (32000, 4, 1), (16000, 2, 2)])
def test_load_audio_shapes_and_content(tmp_path, sr, width, ch):
    n = int(4.0 * sr)
    t = np.arange(n) / sr
    tone = 0.4 * np.sin(2 * np.pi * 440.0 * t)
    x = np.stack([tone] * ch, axis=1)
    p = str(tmp_path / "ref.wav")
    _write(p, x, sr, width, ch)
    y = A.load_audio(p, 32000)
    n32 = -(-n * 32000 // sr)
    assert y.dtype == np.float32 and y.shape == (n32 + 9600,)
    assert np.all(y[n32:] == 0)                                        # 0.3 s of appended silence
    ref = 0.4 * np.sin(2 * np.pi * 440.0 * np.arange(n32) / 32000)
    mid = slice(n32 // 4, 3 * n32 // 4)                                # away from the filter edges
    assert np.max(np.abs(y[mid] - ref[mid])) < 2e-3
    y16 = A.resample(y, 32000, 16000)
    assert y16.shape == (-(-y.shape[0] // 2),)


def test_float_wav_and_errors(tmp_path):
    import struct
    x = (0.25 * np.cos(np.arange(8000) / 10.0)).astype(np.float32)
    p = str(tmp_path / "f.wav")
    data = x.tobytes()
    fmt = struct.pack("<HHIIHH", 3, 1, 16000, 16000 * 4, 4, 32)
    with open(p, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(data)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) + data)
    got, sr = A.read_wav(p)
    assert sr == 16000 and np.array_equal(got[:, 0], x)
    with pytest.raises(ValueError):
        A.read_audio(str(tmp_path / "x.mp3"))


def test_set_reference_audio_bookkeeping(tmp_path):
    from genie_tts_amd import api
    p = str(tmp_path / "clip.wav")
    _write(p, 0.1 * np.random.default_rng(0).standard_normal(3 * 24000), 24000)
    ssl = np.zeros((1, 768, 20), np.float32)
    api.clear_reference_audio_cache()
    api.set_reference_audio("c", p, "テキスト", "ja", phonemes_seq=[3, 96, 222], ssl_content=ssl)
    r = api._reference_audios["c"]
    assert r.audio_32k.shape == (1, 3 * 32000 + 9600) and r.audio_16k.shape == (1, (3 * 32000 + 9600) // 2)
    assert r.phonemes_seq.tolist() == [[3, 96, 222]] and r.text_bert.shape == (3, 1024)
    api.set_reference_audio("d", p, "other", "ja", phonemes_seq=[3, 5])      # cached clip, new text
    assert api._reference_audios["d"] is r and r.phonemes_seq.tolist() == [[3, 5]]
    api.set_reference_audio("e", str(tmp_path / "clip.mp3"), "x", "ja")      # unsupported: logged, ignored
    assert "e" not in api._reference_audios
    with pytest.raises(ValueError):
        api.set_reference_audio("f", p, "x", "klingon", phonemes_seq=[3])
    api.clear_reference_audio_cache()


def _fake_session(monkeypatch, stop_at=None, calls=None):
    """api over a stand-in GENIE.tts: sentence i returns a constant chunk of value i + 1;
    with stop_at = i, stop() arrives while sentence i is synthesized (the stop word is then
    set, and the reference's GENIE.tts returns None, Inference.py:96-97)."""
    from types import SimpleNamespace
    from genie_tts_amd import api
    model = SimpleNamespace(T2S_ENCODER=None, T2S_FIRST_STAGE_DECODER=None, T2S_STAGE_DECODER=None, VITS=None,
                            PROMPT_ENCODER=None, LANGUAGE="Japanese")
    monkeypatch.setattr(api.model_manager, "get", lambda name: model)
    monkeypatch.setitem(api._reference_audios, "stop-c", SimpleNamespace(sv_emb=None))

    def fake_tts(sentence, ref, *a, **k):
        i = int(np.asarray(sentence).reshape(-1)[0])
        if calls is not None:
            calls.append(i)
        if stop_at is not None and i == stop_at:
            api.stop()
        if api.tts_client.stop_event.is_set():
            return None
        return np.full(4, 0.01 * (i + 1), np.float32)

    monkeypatch.setattr(api.tts_client, "tts", fake_tts)
    return api


def _run_async(api, **kw):
    import asyncio

    async def go():
        return [c async for c in api.tts_async("stop-c", None, **kw)]

    return asyncio.run(go())


def test_stop_ends_a_tts_async_session(monkeypatch, tmp_path):
    """TTSPlayer.stop (Core/TTSPlayer.py:208-222): stop() during sentence 2 of a 4-sentence
    tts_async ends the iterator with no further chunk (the worker's chunk_callback(None),
    TTSPlayer.py:109-114 -> Internal.py:258-262) and saves nothing; the next session
    synthesizes every sentence again."""
    calls = []
    api = _fake_session(monkeypatch, stop_at=1, calls=calls)
    monkeypatch.setattr(api, "_sentences", lambda text, split: [np.array([i]) for i in range(4)])
    wav = tmp_path / "s.wav"
    got = _run_async(api, save_path=str(wav))
    assert len(got) == 1 and calls == [0, 1] and not wav.exists()
    assert np.frombuffer(got[0], np.int16)[0] == int(0.01 * 32767)
    calls.clear()
    monkeypatch.setattr(api.tts_client, "tts", _fake_session(monkeypatch, calls=calls).tts_client.tts)
    again = _run_async(api, save_path=str(wav))
    assert len(again) == 4 and calls == [0, 1, 2, 3] and wav.exists()


def test_stop_ends_a_tts_session(monkeypatch, tmp_path):
    """api.tts: the sentences before the stop are returned, none after it, nothing is saved;
    a stop() issued before a session does not leak into it."""
    calls = []
    api = _fake_session(monkeypatch, stop_at=2, calls=calls)
    monkeypatch.setattr(api, "_sentences", lambda text, split: [np.array([i]) for i in range(5)])
    monkeypatch.setattr(api, "_synthesize_all",
                        lambda name, ss, tb, sp: [api._synthesize(name, s, tb, sp) for s in ss])
    wav = tmp_path / "t.wav"
    out = api.tts("stop-c", None, save_path=str(wav))
    assert calls == [0, 1, 2] and out.shape == (8,) and not wav.exists()
    calls.clear()
    api.stop()                                  # between sessions
    api2 = _fake_session(monkeypatch, calls=calls)
    out = api2.tts("stop-c", None, save_path=str(wav))
    assert calls == [0, 1, 2, 3, 4] and out.shape == (20,) and wav.exists()
