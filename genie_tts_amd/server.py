"""HTTP server: the reference's FastAPI app (src/genie_tts/Server.py:22-175), same
endpoints and payloads, served as a front router over N engine worker processes
pinned one per GPU (the reference runs one uvicorn worker with one
CPU ONNX session set, and uvicorn `workers > 1` cannot share its globals).

  POST /load_character, /unload_character, /set_reference_audio,
       /clear_reference_audio_cache   -> broadcast to every worker (each GPU holds
                                          every character: replicas, no collective)
  POST /tts                           -> the least-loaded worker; StreamingResponse of
                                          raw 16-bit PCM, one chunk per sentence, as
                                          the reference's TTSPlayer chunk callback
                                          (Server.py:122-143, TTSPlayer.py:98-107)
  POST /stop                          -> every worker

A worker is a spawned process with HIP_VISIBLE_DEVICES set before anything touches
the GPU.  It batches the requests waiting for it: the next sentence of every
pending request (same character) goes through ONE batched T2S (packed prefill +
ragged decode) and the concurrent vocoder lanes, so a burst of requests shares
weight reads instead of queueing one utterance at a time; each sentence's PCM is
sent back as soon as its batch is done.  G2P / CN-HuBERT / SV stay outside the
engine: workers import them from `module:function` specs (set_g2p et al.).
"""


import asyncio
import importlib
import itertools
import logging
import multiprocessing as mp
import os
import threading
import time
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

MAX_BATCH = 64


def _resolve(spec: Optional[str]):
    if not spec:
        return None
    mod, _, fn = spec.partition(":")
    return getattr(importlib.import_module(mod), fn)


def round_size(ready: int) -> int:
    """Sentences a worker round takes out of `ready` of one character: all of them, up to
    MAX_BATCH.  The T2S time per batch grows monotonically and slowly with B
    (tools/batch_sweep.py, profiles/r03i_batch_sweep.json: 16.7 ms at 1, 27 ms at 8,
    69 ms at 32, 129 ms at 64 per 81-step generate), so a round never waits."""
    return min(ready, MAX_BATCH)


# --------------------------------------------------------------------- worker
def _worker_main(index: int, conn, cfg: dict) -> None:
    """One GPU (HIP_VISIBLE_DEVICES was set by the router before spawning)."""
    import numpy as np
    import genie_tts_amd as genie
    from genie_tts_amd import api, audio as A
    from genie_tts_amd.engine import make_sampler
    from genie_tts_amd.inference import tts_client
    from genie_tts_amd.model_manager import model_manager
    from genie_tts_amd.text_splitter import TextSplitter

    genie.set_g2p(_resolve(cfg.get("g2p")))
    genie.set_ssl_extractor(_resolve(cfg.get("ssl")))
    genie.set_sv_extractor(_resolve(cfg.get("sv")))
    if cfg.get("greedy"):
        model_manager.sampler = make_sampler(greedy=True)
    if cfg.get("noise"):             # "zero": deterministic vocoder noise (tests pin the streamed audio)
        model_manager.vits_noise = cfg["noise"]
    splitter = TextSplitter()
    pipeline = bool(cfg.get("pipeline", False))
    pending: List[dict] = []        # tts requests: {"id", "character_name", "sentences", "next", "force_steps"}

    def reply(**kw):
        conn.send(kw)

    def control(msg) -> None:
        cmd = msg["cmd"]
        finish_inflight()            # control calls may replace what the overlapped vocoder uses
        try:
            if cmd == "load_character":
                genie.load_character(msg["character_name"], msg["onnx_model_dir"], msg["language"])
            elif cmd == "load_synthetic":
                from genie_tts_amd import synth
                genie.load_weights(msg["character_name"], synth.synthetic_character(msg.get("version", "v2")),
                                   msg.get("version", "v2"), msg.get("language", "Japanese"))
            elif cmd == "unload_character":
                genie.unload_character(msg["character_name"])
            elif cmd == "set_reference_audio":
                genie.set_reference_audio(msg["character_name"], msg["audio_path"], msg["audio_text"],
                                          msg["language"])
                if msg["character_name"] not in api._reference_audios:
                    raise ValueError("reference audio rejected (see worker log)")
            elif cmd == "clear_reference_audio_cache":
                genie.clear_reference_audio_cache()
            elif cmd == "stop":
                genie.stop()
                for r in pending:
                    reply(kind="end", id=r["id"])
                pending.clear()
            reply(kind="ok", id=msg["id"])
        except Exception as e:       # noqa: BLE001 -- reported to the router as HTTP 500
            reply(kind="error", id=msg["id"], detail=f"{type(e).__name__}: {e}")

    def accept(msg) -> None:
        text = msg["text"]
        sents = splitter.split(text.strip()) if msg.get("split_sentence") else [text]
        sents = [s for s in sents if s]
        if not sents:
            reply(kind="end", id=msg["id"])
            return
        pending.append({"id": msg["id"], "character_name": msg["character_name"], "sentences": sents, "next": 0,
                        "force_steps": int(msg.get("force_steps") or 0), "save_path": msg.get("save_path"),
                        "chunks": []})

    inflight: List[tuple] = []      # [(group, sentence indexes, wavs, engine)] of the overlapped vocoder

    def finish_inflight() -> None:
        """Join the overlapped vocoder of the previous round and stream its chunks."""
        if not inflight:
            return
        group, idx, wavs, eng = inflight.pop()
        try:
            if eng is not None:
                eng.vits_batch_wait()
            wavs = [w if isinstance(w, np.ndarray) else w.cpu().numpy() for w in wavs]
        except Exception as e:       # noqa: BLE001
            for r in group:
                reply(kind="error", id=r["id"], detail=f"{type(e).__name__}: {e}")
                if r in pending:
                    pending.remove(r)
            return
        for r, i, wav in zip(group, idx, wavs):
            if r not in pending:      # failed or stopped meanwhile
                continue
            reply(kind="chunk", id=r["id"], data=A.to_pcm16(wav))
            r["chunks"].append(np.asarray(wav, np.float32).reshape(-1))
            r["done"] = i + 1
            if r["done"] == len(r["sentences"]):
                pending.remove(r)
                if r["save_path"]:
                    try:              # a client-supplied path: its failure ends this request only
                        A.write_wav(r["save_path"], np.concatenate(r["chunks"]))
                    except Exception as e:   # noqa: BLE001
                        reply(kind="error", id=r["id"], detail=f"save_path: {type(e).__name__}: {e}")
                        continue
                reply(kind="end", id=r["id"])

    def run_round() -> None:
        """The next sentence of up to MAX_BATCH pending requests of one character.  With
        cfg["pipeline"] this round's T2S runs beside the previous round's vocoder
        (gsv_vits_decode_batch_async), whose chunks are streamed once this T2S is done; with
        nothing left to start, the vocoder is joined at once.  Off by default: measured on
        one MI355X it raised p50 first audio (50 QPS: 47 -> 58 ms) without raising the
        saturated rate (profiles/r02g_server_qps_pipeline.json)."""
        ready = [r for r in pending if r["next"] < len(r["sentences"])]
        if not ready:
            finish_inflight()
            return
        name = ready[0]["character_name"]
        group = [r for r in ready if r["character_name"] == name]
        group = group[:round_size(len(group))]
        idx = [r["next"] for r in group]
        try:
            m = model_manager.get(name)
            ref = api._reference_audios.get(name)
            if m is None or ref is None:
                raise ValueError("Character not found or reference audio not set.")
            items = []
            for r in group:
                ts, tb = api._g2p("。" + r["sentences"][r["next"]], m.LANGUAGE)      # Inference.py:27-28
                items.append((ts, tb, r["force_steps"]))
            tts_client.stop_event.clear()
            toks = tts_client.tts_batch_t2s(items, ref, m, m.T2S_FIRST_STAGE_DECODER.sampler)
            finish_inflight()
            eng = m.ENGINE if getattr(m.VITS, "engine", None) is m.ENGINE else None
            overlapped = pipeline and eng is not None
            wavs = tts_client.tts_batch_vocoder(items, toks, ref, m, overlapped=overlapped)
        except Exception as e:       # noqa: BLE001
            finish_inflight()
            for r in group:
                reply(kind="error", id=r["id"], detail=f"{type(e).__name__}: {e}")
                if r in pending:
                    pending.remove(r)
            return
        for r in group:
            r["next"] += 1
        inflight.append((group, idx, wavs, eng if overlapped else None))
        if not overlapped:
            finish_inflight()

    def fail_all(e: Exception) -> None:
        """An unexpected error outside a request's own handler: every request in this
        worker gets an error reply and the worker keeps serving."""
        logger.exception("worker %d: round failed", index)
        inflight.clear()
        for r in pending:
            reply(kind="error", id=r["id"], detail=f"worker error: {type(e).__name__}: {e}")
        pending.clear()

    reply(kind="ready", id=-1, index=index)
    while True:
        # block only when idle; otherwise drain what has arrived, then run one round
        while (not pending and not inflight) or conn.poll():
            msg = conn.recv()
            if msg is None:
                return
            try:
                if msg["cmd"] == "tts":
                    accept(msg)
                else:
                    control(msg)
            except Exception as e:   # noqa: BLE001
                fail_all(e)
            if pending and not conn.poll():
                break
        try:
            run_round()
        except Exception as e:   # noqa: BLE001
            fail_all(e)


# --------------------------------------------------------------------- router
class Router:
    """Owns the worker processes; never touches the GPU itself."""

    def __init__(self, gpus: List[int], g2p: Optional[str] = None, ssl: Optional[str] = None,
                 sv: Optional[str] = None, greedy: bool = False, worker=None, pipeline: bool = False,
                 noise: Optional[str] = None):
        self.gpus = gpus
        self.worker = worker or _worker_main         # tests substitute a host-only worker
        self.cfg = {"g2p": g2p, "ssl": ssl, "sv": sv, "greedy": greedy, "pipeline": pipeline, "noise": noise}
        self.ids = itertools.count(1)
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.queues: Dict[int, asyncio.Queue] = {}
        self.load: List[int] = [0] * len(gpus)
        self.conns, self.procs, self.threads = [], [], []
        self.send_locks: List[threading.Lock] = []
        self.dead: set = set()                        # workers whose pipe closed
        self.sent_to: Dict[int, set] = {}             # request id -> workers that owe it replies
        self.state_lock = threading.Lock()

    def start(self, loop: asyncio.AbstractEventLoop, timeout: float = 600.0) -> None:
        self.loop = loop
        ctx = mp.get_context("spawn")
        saved = os.environ.get("HIP_VISIBLE_DEVICES")
        ready = []
        for i, g in enumerate(self.gpus):
            parent, child = ctx.Pipe()
            os.environ["HIP_VISIBLE_DEVICES"] = str(g)     # inherited by the spawned interpreter
            p = ctx.Process(target=self.worker, args=(i, child, self.cfg), daemon=True)
            p.start()
            self.conns.append(parent)
            self.procs.append(p)
            self.send_locks.append(threading.Lock())
        if saved is None:
            os.environ.pop("HIP_VISIBLE_DEVICES", None)
        else:
            os.environ["HIP_VISIBLE_DEVICES"] = saved
        for i, c in enumerate(self.conns):
            if not c.poll(timeout):
                raise RuntimeError(f"worker {i} did not start")
            ready.append(c.recv())
        for i, c in enumerate(self.conns):
            t = threading.Thread(target=self._reader, args=(i, c), daemon=True)
            t.start()
            self.threads.append(t)

    def _reader(self, i: int, conn) -> None:
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                self._worker_died(i)
                return
            if msg.get("kind") != "chunk":   # a final reply: worker i owes this request nothing more
                with self.state_lock:
                    ws = self.sent_to.get(msg["id"])
                    if ws is not None:
                        ws.discard(i)
            q = self.queues.get(msg["id"])
            if q is not None:
                self.loop.call_soon_threadsafe(q.put_nowait, (i, msg))

    def _worker_died(self, i: int) -> None:
        """Worker i's pipe closed: it gets no more requests, and every request still
        waiting on it (a tts stream or a broadcast's reply) gets an error."""
        with self.state_lock:
            self.dead.add(i)
            owed = [rid for rid, ws in self.sent_to.items() if i in ws]
        if not getattr(self, "closing", False):
            logger.error("worker %d exited; %d request(s) failed", i, len(owed))
        for rid in owed:
            q = self.queues.get(rid)
            if q is not None:
                self.loop.call_soon_threadsafe(q.put_nowait, (i, dict(kind="error", id=rid,
                                                                     detail=f"worker {i} exited")))

    def _send(self, i: int, msg: dict) -> None:
        with self.send_locks[i]:
            self.conns[i].send(msg)

    def _live(self) -> List[int]:
        with self.state_lock:
            live = [i for i in range(len(self.conns)) if i not in self.dead]
        if not live:
            raise RuntimeError("no live engine worker")
        return live

    async def broadcast(self, cmd: str, **kw) -> List[dict]:
        rid = next(self.ids)
        q: asyncio.Queue = asyncio.Queue()
        self.queues[rid] = q
        try:
            live = self._live()
            with self.state_lock:
                self.sent_to[rid] = set(live)
            for i in live:
                self._send(i, dict(cmd=cmd, id=rid, **kw))
            got: Dict[int, dict] = {}
            while len(got) < len(live):         # one reply per worker (a dying worker's error
                i, msg = await q.get()          # may follow its own final reply: keep the first)
                got.setdefault(i, msg)
            return [got[i] for i in live]
        finally:
            self.queues.pop(rid, None)
            with self.state_lock:
                self.sent_to.pop(rid, None)

    async def tts(self, **kw):
        """Async iterator of PCM chunks from the least-loaded live worker."""
        rid = next(self.ids)
        q: asyncio.Queue = asyncio.Queue()
        self.queues[rid] = q
        # pick the worker and record what it owes under one lock: a worker that dies before
        # is not picked, one that dies after finds this request in sent_to (_worker_died)
        with self.state_lock:
            live = [k for k in range(len(self.conns)) if k not in self.dead]
            if not live:
                self.queues.pop(rid, None)
                raise RuntimeError("no live engine worker")
            i = min(live, key=lambda k: self.load[k])
            self.load[i] += 1
            self.sent_to[rid] = {i}
        try:
            self._send(i, dict(cmd="tts", id=rid, **kw))
            while True:
                _, msg = await q.get()
                if msg["kind"] == "chunk":
                    yield msg["data"]
                elif msg["kind"] == "error":
                    raise RuntimeError(msg["detail"])
                else:
                    return
        finally:
            self.load[i] -= 1
            self.queues.pop(rid, None)
            with self.state_lock:
                self.sent_to.pop(rid, None)

    def close(self) -> None:
        self.closing = True
        for i, c in enumerate(self.conns):
            try:
                self._send(i, None)
            except Exception:   # noqa: BLE001
                pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()


def create_app(router: Router):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import StreamingResponse
    from pydantic import BaseModel

    from .api import SUPPORTED_AUDIO_EXTS, _norm_language

    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(_app):
        if router.loop is None:
            router.start(asyncio.get_running_loop())
        yield

    app = FastAPI(lifespan=lifespan)

    class CharacterPayload(BaseModel):
        character_name: str
        onnx_model_dir: str
        language: str

    class UnloadCharacterPayload(BaseModel):
        character_name: str

    class ReferenceAudioPayload(BaseModel):
        character_name: str
        audio_path: str
        audio_text: str
        language: str

    class TTSPayload(BaseModel):
        character_name: str
        text: str
        split_sentence: bool = False
        save_path: Optional[str] = None
        force_steps: int = 0          # benchmark knob (random weights never emit EOS); 0 = the reference's rule

    def check(res: List[dict]) -> None:
        bad = [r for r in res if r["kind"] == "error"]
        if bad:
            raise HTTPException(status_code=500, detail=bad[0]["detail"])

    @app.post("/load_character")
    async def load_character_endpoint(payload: CharacterPayload):
        check(await router.broadcast("load_character", character_name=payload.character_name,
                                     onnx_model_dir=payload.onnx_model_dir, language=payload.language))
        return {"status": "success", "message": f"Character '{payload.character_name}' loaded."}

    @app.post("/unload_character")
    async def unload_character_endpoint(payload: UnloadCharacterPayload):
        check(await router.broadcast("unload_character", character_name=payload.character_name))
        return {"status": "success", "message": f"Character '{payload.character_name}' unloaded."}

    @app.post("/set_reference_audio")
    async def set_reference_audio_endpoint(payload: ReferenceAudioPayload):
        ext = os.path.splitext(payload.audio_path)[1].lower()
        if ext not in SUPPORTED_AUDIO_EXTS:
            raise HTTPException(status_code=400, detail=f"Audio format '{ext}' is not supported. "
                                                        f"Supported formats: {sorted(SUPPORTED_AUDIO_EXTS)}")
        check(await router.broadcast("set_reference_audio", character_name=payload.character_name,
                                     audio_path=payload.audio_path, audio_text=payload.audio_text,
                                     language=_norm_language(payload.language)))
        return {"status": "success", "message": f"Reference audio for '{payload.character_name}' set."}

    @app.post("/tts")
    async def tts_endpoint(payload: TTSPayload):
        gen = router.tts(character_name=payload.character_name, text=payload.text,
                         split_sentence=payload.split_sentence, save_path=payload.save_path,
                         force_steps=payload.force_steps)
        try:    # surface "not found" as 404 before the stream starts, as the reference does
            first = await gen.__anext__()
        except StopAsyncIteration:
            first = None
        except RuntimeError as e:
            code = 404 if "not found" in str(e) else 500
            raise HTTPException(status_code=code, detail=str(e))

        async def body():
            if first is not None:
                yield first
                async for c in gen:
                    yield c
        return StreamingResponse(body(), media_type="audio/wav")

    @app.post("/stop")
    async def stop_endpoint():
        check(await router.broadcast("stop"))
        return {"status": "success", "message": "TTS stopped."}

    @app.post("/clear_reference_audio_cache")
    async def clear_reference_audio_cache_endpoint():
        check(await router.broadcast("clear_reference_audio_cache"))
        return {"status": "success", "message": "Reference audio cache cleared."}

    return app


def start_server(host: str = "127.0.0.1", port: int = 8000, gpus: Optional[List[int]] = None,
                 g2p: Optional[str] = None, ssl: Optional[str] = None, sv: Optional[str] = None) -> None:
    """Server.py:174-175 with one engine worker per GPU instead of uvicorn workers."""
    import uvicorn
    if gpus is None:
        n = int(os.environ.get("GENIE_GPUS", "1"))
        gpus = list(range(n))
    router = Router(gpus, g2p=g2p, ssl=ssl, sv=sv)
    try:
        uvicorn.run(create_app(router), host=host, port=port, workers=1)
    finally:
        router.close()


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("GENIE_GPUS", "1")))
    ap.add_argument("--g2p")
    ap.add_argument("--ssl")
    ap.add_argument("--sv")
    a = ap.parse_args()
    start_server(a.host, a.port, list(range(a.gpus)), a.g2p, a.ssl, a.sv)
