"""GPU: the HTTP server end to end -- FastAPI router + one engine worker process on
the GPU (genie_tts_amd/server.py), a synthetic V2 character and a reference WAV set
through the reference's endpoints; concurrent /tts requests with sentence
splitting are batched by the worker and streamed back one 16-bit PCM chunk per
sentence (Server.py:122-143).  With greedy sampling and zero vocoder noise every
streamed sentence is checked against the CPU oracle (oracle/restate.py) fed what the
worker is fed (the same WAV reader / resampler, G2P and SSL stand-ins): int16 PCM
within one step, audio RMS <= 1e-4."""
import asyncio
import wave

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(wav_path, ref_text, G):
    """sentence -> the oracle's audio for it, from what the worker computes on its host
    side: audio.load_audio / resample of the reference WAV (set_reference_audio), the
    toy G2P of the reference text and of '。' + sentence (Inference.py:27), toy SSL."""
    import torch
    from genie_tts_amd import audio as A, stubs
    from oracle import restate as R
    from tests.common import character
    torch.set_num_threads(8)
    w = character("v2")
    m = R.T2SModel(w["t2s"])
    vm = R.VitsModel(w["vits"], "v2")
    a32 = A.load_audio(wav_path, 32000).reshape(1, -1)
    ssl = stubs.toy_ssl(A.resample(a32[0], 32000, 16000).reshape(1, -1))
    ps, rb = stubs.toy_g2p(ref_text, "Japanese")

    def sentence(s):
        ts, tb = stubs.toy_g2p("。" + s, "Japanese")
        sem, _, _ = R.t2s_generate(w["t2s_encoder"], m, ps, rb, ts, tb, ssl, force_steps=G + 1)
        return vm(ts, np.asarray(sem).reshape(1, 1, -1), ref_audio=a32).numpy().reshape(-1)
    return sentence


@pytest.mark.parametrize("pipeline", [False, True])
def test_server_concurrent_streams(tmp_path, pipeline):
    """pipeline=True: each round's vocoder beside the next round's T2S (the chunks of a
    round are streamed after the next round's T2S; same sizes, same order)."""
    import httpx
    from genie_tts_amd.server import Router, create_app
    from genie_tts_amd.text_splitter import TextSplitter
    wav = str(tmp_path / "ref.wav")
    x = (0.1 * np.random.default_rng(1).standard_normal(4 * 32000)).clip(-1, 1)
    with wave.open(wav, "wb") as wf:
        wf.setnchannels(1); wf.setsampwidth(2); wf.setframerate(32000)
        wf.writeframes((x * 32767).astype("<i2").tobytes())
    texts = ["今日はいい天気ですね。散歩に行きましょう！", "ありがとうございます。", "また明日会いましょう。元気でね！"]
    G = 24
    oracle_sentence = _oracle(wav, "こんにちは。", G)

    async def run():
        router = Router([0], g2p="genie_tts_amd.stubs:toy_g2p", ssl="genie_tts_amd.stubs:toy_ssl", greedy=True,
                        pipeline=pipeline, noise="zero")
        router.start(asyncio.get_running_loop(), timeout=300)
        try:
            res = await router.broadcast("load_synthetic", character_name="srv", version="v2")
            assert all(r["kind"] == "ok" for r in res), res
            tr = httpx.ASGITransport(app=create_app(router))
            async with httpx.AsyncClient(transport=tr, base_url="http://t", timeout=300) as cl:
                r = await cl.post("/set_reference_audio", json=dict(character_name="srv", audio_path=wav,
                                                                    audio_text="こんにちは。", language="ja"))
                assert r.status_code == 200, r.text

                async def one(t):
                    chunks = []
                    async with cl.stream("POST", "/tts", json=dict(character_name="srv", text=t,
                                                                   split_sentence=True, force_steps=G + 1)) as s:
                        assert s.status_code == 200
                        async for c in s.aiter_bytes():
                            chunks.append(c)
                    return b"".join(chunks)
                outs = await asyncio.gather(*[one(t) for t in texts])
                for t, o in zip(texts, outs):
                    sents = TextSplitter().split(t)
                    pcm = np.frombuffer(o, np.int16)
                    assert pcm.size == len(sents) * 1280 * G
                    for i, s in enumerate(sents):
                        want = oracle_sentence(s)
                        got = pcm[i * 1280 * G:(i + 1) * 1280 * G]
                        assert np.abs(got.astype(np.int32) - (want * 32767).astype(np.int16)).max() <= 1, (t, i)
                        rms = float(np.sqrt(np.mean((got / 32767.0 - want) ** 2)))
                        assert rms <= 1e-4, (t, i, rms)
                r = await cl.post("/tts", json=dict(character_name="nobody", text="x"))
                assert r.status_code == 404
        finally:
            router.close()
    asyncio.run(run())
