"""CPU: the server's router (genie_tts_amd/server.py) -- the reference's endpoints
(Server.py:46-165) over 2 spawned worker processes, broadcast of control calls,
least-loaded dispatch, per-sentence streaming of raw PCM and the 404 of an unknown
character -- with a host-only worker (the engine worker needs a GPU; its batching
is covered by tests/test_server_gpu.py)."""
import asyncio
import os

import numpy as np
import pytest


def fake_worker(index, conn, cfg):
    """Replies like _worker_main: one PCM chunk per sentence, value = worker index."""
    from genie_tts_amd.text_splitter import TextSplitter
    chars = set()
    conn.send(dict(kind="ready", id=-1, index=index))
    while True:
        msg = conn.recv()
        if msg is None:
            return
        if msg["cmd"] == "tts":
            if msg["character_name"] not in chars:
                conn.send(dict(kind="error", id=msg["id"], detail="Character not found or reference audio not set."))
                continue
            sents = TextSplitter().split(msg["text"]) if msg["split_sentence"] else [msg["text"]]
            for s in sents:
                conn.send(dict(kind="chunk", id=msg["id"], data=np.full(len(s), index, np.int16).tobytes()))
            conn.send(dict(kind="end", id=msg["id"]))
        else:
            if msg["cmd"] == "set_reference_audio":
                chars.add(msg["character_name"])
            conn.send(dict(kind="ok", id=msg["id"]))


def test_router_endpoints_and_streaming(tmp_path):
    import httpx
    from genie_tts_amd.server import Router, create_app

    async def run():
        router = Router([0, 1], worker=fake_worker)
        router.start(asyncio.get_running_loop(), timeout=120)
        app = create_app(router)
        tr = httpx.ASGITransport(app=app)
        try:
            async with httpx.AsyncClient(transport=tr, base_url="http://t") as cl:
                r = await cl.post("/tts", json=dict(character_name="a", text="x"))
                assert r.status_code == 404
                r = await cl.post("/set_reference_audio", json=dict(character_name="a", audio_path="r.mp3",
                                                                    audio_text="t", language="ja"))
                assert r.status_code == 400
                r = await cl.post("/set_reference_audio", json=dict(character_name="a", audio_path="r.wav",
                                                                    audio_text="t", language="ja"))
                assert r.status_code == 200 and r.json()["status"] == "success"
                text = "今日はいい天気ですね。散歩に行きましょう！"

                async def one():
                    r = await cl.post("/tts", json=dict(character_name="a", text=text, split_sentence=True))
                    assert r.status_code == 200
                    return np.frombuffer(r.content, np.int16)
                outs = await asyncio.gather(*[one() for _ in range(8)])
                from genie_tts_amd.text_splitter import TextSplitter
                assert all(o.size == sum(len(s) for s in TextSplitter().split(text)) for o in outs)
                workers = {int(o[0]) for o in outs}
                assert workers == {0, 1}                      # load spread over both workers
                for name in ("stop", "clear_reference_audio_cache"):
                    assert (await cl.post("/" + name)).status_code == 200
        finally:
            router.close()
    asyncio.run(run())


def test_round_size_policy():
    from genie_tts_amd.server import MAX_BATCH, round_size
    assert [round_size(n) for n in range(1, 12)] == [1, 2, 3, 4, 4, 4, 4, 4, 4, 10, 11]
    assert round_size(200) == MAX_BATCH
