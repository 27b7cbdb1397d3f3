"""GPU: the HTTP server end to end -- FastAPI router + one engine worker process on
the GPU (genie_tts_amd/server.py), a synthetic V2 character and a reference WAV set
through the reference's endpoints; concurrent /tts requests with sentence
splitting are batched by the worker and streamed back one 16-bit PCM chunk per
sentence (Server.py:122-143)."""
import asyncio
import wave

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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

    async def run():
        router = Router([0], g2p="genie_tts_amd.stubs:toy_g2p", ssl="genie_tts_amd.stubs:toy_ssl", greedy=True,
                        pipeline=pipeline)
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
                    n = len(TextSplitter().split(t))
                    pcm = np.frombuffer(o, np.int16)
                    assert pcm.size == n * 1280 * G
                    assert np.abs(pcm).max() > 0
                r = await cl.post("/tts", json=dict(character_name="nobody", text="x"))
                assert r.status_code == 404
        finally:
            router.close()
    asyncio.run(run())
