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
    assert [round_size(n) for n in range(1, 12)] == list(range(1, 12))
    assert round_size(200) == MAX_BATCH


def _host_worker_env(monkeypatch):
    """_worker_main's engine calls replaced by host stand-ins (one float per sentence
    index), so its request bookkeeping runs on the CPU in a thread."""
    from genie_tts_amd import api
    from genie_tts_amd.inference import tts_client
    from genie_tts_amd.model_manager import model_manager

    class M:
        LANGUAGE = "Japanese"
        ENGINE = None
        VITS = None
        T2S_FIRST_STAGE_DECODER = type("D", (), {"sampler": None})()

    monkeypatch.setattr(model_manager, "get", lambda name: M() if name == "a" else None)
    monkeypatch.setitem(api._reference_audios, "a", object())
    monkeypatch.setattr(tts_client, "tts_batch_t2s", lambda items, ref, m, sp: [None] * len(items))
    monkeypatch.setattr(tts_client, "tts_batch_vocoder",
                        lambda items, toks, ref, m, overlapped=False: [np.full(8, 0.25, np.float32) for _ in items])


def _collect(conn, rid):
    kinds = []
    while True:
        assert conn.poll(60), "worker did not answer"
        m = conn.recv()
        if m["id"] != rid:
            continue
        kinds.append(m["kind"])
        if m["kind"] in ("end", "error"):
            return kinds, m


def test_worker_survives_unwritable_save_path(tmp_path, monkeypatch):
    """a client save_path that cannot be written ends THAT request with an
    error reply (after its chunks); the worker keeps serving the next request."""
    import multiprocessing as mp
    import threading
    from genie_tts_amd import api
    from genie_tts_amd.server import _worker_main
    _host_worker_env(monkeypatch)
    blocker = tmp_path / "file"
    blocker.write_text("x")                       # a regular file: no directory can be made under it
    parent, child = mp.Pipe()
    t = threading.Thread(target=_worker_main, args=(0, child, {"g2p": "genie_tts_amd.stubs:toy_g2p"}),
                         daemon=True)
    t.start()
    try:
        assert parent.poll(60) and parent.recv()["kind"] == "ready"
        from genie_tts_amd.text_splitter import TextSplitter
        text = "今日はいい天気ですね。散歩に行きましょう！"
        n = len(TextSplitter().split(text))
        assert n == 2
        parent.send(dict(cmd="tts", id=1, character_name="a", text=text, split_sentence=True,
                         save_path=str(blocker / "sub" / "out.wav")))
        kinds, last = _collect(parent, 1)
        assert kinds == ["chunk"] * n + ["error"] and "save_path" in last["detail"], (kinds, last)
        good = tmp_path / "ok.wav"
        parent.send(dict(cmd="tts", id=2, character_name="a", text="かき。", split_sentence=True,
                         save_path=str(good)))
        kinds, _ = _collect(parent, 2)
        assert kinds == ["chunk", "end"] and good.exists()
        parent.send(dict(cmd="tts", id=3, character_name="nobody", text="x"))
        kinds, last = _collect(parent, 3)
        assert kinds == ["error"] and "not found" in last["detail"]
    finally:
        parent.send(None)
        t.join(timeout=30)
        api.set_g2p(None)


def dying_worker(index, conn, cfg):
    """Worker 0 exits on its first tts request (a crashed GPU process); worker 1 serves."""
    conn.send(dict(kind="ready", id=-1, index=index))
    while True:
        msg = conn.recv()
        if msg is None:
            return
        if msg["cmd"] == "tts":
            if index == 0:
                os._exit(3)
            conn.send(dict(kind="chunk", id=msg["id"], data=np.full(4, index, np.int16).tobytes()))
            conn.send(dict(kind="end", id=msg["id"]))
        else:
            conn.send(dict(kind="ok", id=msg["id"]))


def test_router_fails_requests_of_a_dead_worker():
    """when a worker's pipe closes, its in-flight requests fail instead of
    hanging, and later requests and broadcasts go to the live workers only."""
    from genie_tts_amd.server import Router

    async def run():
        router = Router([0, 1], worker=dying_worker)
        router.start(asyncio.get_running_loop(), timeout=120)
        try:
            async def one():
                return b"".join([c async for c in router.tts(character_name="a", text="x")])
            with pytest.raises(RuntimeError, match="exited"):
                await asyncio.wait_for(one(), 60)       # least-loaded: worker 0, which dies
            for _ in range(3):
                out = await asyncio.wait_for(one(), 60)
                assert np.frombuffer(out, np.int16).tolist() == [1, 1, 1, 1]
            res = await asyncio.wait_for(router.broadcast("stop"), 60)
            assert [r["kind"] for r in res] == ["ok"]
        finally:
            router.close()
    asyncio.run(run())


def reply_then_die_worker(index, conn, cfg):
    """Worker 0 answers the 'stop' broadcast and then exits; worker 1 answers it late."""
    import time
    conn.send(dict(kind="ready", id=-1, index=index))
    while True:
        msg = conn.recv()
        if msg is None:
            return
        if index == 1:
            time.sleep(0.5)
        conn.send(dict(kind="ok", id=msg["id"], index=index))
        if index == 0:
            conn.close()
            os._exit(0)


def test_broadcast_keeps_the_reply_of_a_worker_that_dies_after_answering():
    """a worker's final reply clears what it owes, so its later death adds no
    error for that request, and a broadcast waits for one reply from every worker."""
    from genie_tts_amd.server import Router

    async def run():
        router = Router([0, 1], worker=reply_then_die_worker)
        router.start(asyncio.get_running_loop(), timeout=120)
        try:
            res = await asyncio.wait_for(router.broadcast("stop"), 60)
            assert [(r["kind"], r.get("index")) for r in res] == [("ok", 0), ("ok", 1)]
        finally:
            router.close()
    asyncio.run(run())
