"""configs[4]: the HTTP server (genie_tts_amd/server.py: FastAPI router + one engine
worker per GPU) under a concurrent open-loop load: Poisson arrivals at a swept QPS,
each request one 20-character JP sentence streamed back as 16-bit PCM; reports p50 /
p90 / p99 first-audio latency (request sent -> first PCM byte) and the achieved
throughput.  Synthetic V2 character (seeded weights, no checkpoints offline), toy
G2P / SSL stand-ins (genie_tts_amd/stubs.py); every sentence is forced to 81 loop
steps = 80 semantic tokens = 3.2 s of audio (random weights never emit EOS).

Usage: python tools/qps_sweep.py [--gpus N] [--qps 5,10,20,40,80] [--requests 1000] [--pipeline 0|1]
Prints one JSON line.
"""
import argparse
import asyncio
import json
import os
import sys
import time
import wave

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sentences(n, seed=7):
    r = np.random.default_rng(seed)
    kana = [chr(c) for c in range(0x3042, 0x3094)]
    return ["".join(r.choice(kana, 19)) + "。" for _ in range(n)]


async def main():
    import httpx
    import uvicorn
    from genie_tts_amd.server import Router, create_app
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--qps", default="5,10,20,40,80,160")
    ap.add_argument("--requests", type=int, default=1000)
    ap.add_argument("--port", type=int, default=8765)
    ap.add_argument("--pipeline", type=int, default=0,
                    help="workers overlap each round's vocoder with the next round's T2S")
    a = ap.parse_args()

    router = Router(list(range(a.gpus)), g2p="genie_tts_amd.stubs:toy_g2p", ssl="genie_tts_amd.stubs:toy_ssl",
                    greedy=True, pipeline=bool(a.pipeline))
    loop = asyncio.get_running_loop()
    t0 = time.time()
    router.start(loop)
    app = create_app(router)
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=a.port, log_level="warning"))
    srv = asyncio.create_task(server.serve())
    while not server.started:
        await asyncio.sleep(0.05)
    # a synthetic character on every worker + a reference clip
    res = await router.broadcast("load_synthetic", character_name="bench", version="v2")
    assert all(r["kind"] == "ok" for r in res), res
    wav = "/tmp/genie_qps_ref.wav"
    x = (0.1 * np.random.default_rng(3).standard_normal(int(5.0 * 32000))).clip(-1, 1)
    with wave.open(wav, "wb") as wf:
        wf.setnchannels(1); wf.setsampwidth(2); wf.setframerate(32000)
        wf.writeframes((x * 32767).astype("<i2").tobytes())
    base = f"http://127.0.0.1:{a.port}"
    async with httpx.AsyncClient(timeout=600.0) as cl:
        r = await cl.post(base + "/set_reference_audio", json=dict(character_name="bench", audio_path=wav,
                                                                    audio_text="こんにちは。", language="ja"))
        assert r.status_code == 200, r.text
        startup_s = time.time() - t0

        async def one(text, lat, done):
            t = time.perf_counter()
            first = None
            n = 0
            async with cl.stream("POST", base + "/tts", json=dict(character_name="bench", text=text,
                                                                  force_steps=81)) as resp:
                assert resp.status_code == 200
                async for chunk in resp.aiter_bytes():
                    if first is None:
                        first = time.perf_counter() - t
                    n += len(chunk)
            lat.append(first)
            done.append((time.perf_counter() - t, n))

        # warm-up: the engines build their decode graphs / workspaces
        for k in (1, 8, 32):
            await asyncio.gather(*[one(s, [], []) for s in sentences(k, 99 + k)])
        out = []
        for qps in [float(q) for q in a.qps.split(",")]:
            texts = sentences(a.requests, int(qps * 10))
            gaps = np.random.default_rng(int(qps)).exponential(1.0 / qps, size=len(texts))
            lat, done, tasks = [], [], []
            t_start = time.perf_counter()
            t_note = time.perf_counter()
            for k, (text, g) in enumerate(zip(texts, gaps)):
                tasks.append(asyncio.create_task(one(text, lat, done)))
                await asyncio.sleep(g)
                if time.perf_counter() - t_note > 30:   # progress (long low-QPS points)
                    print(f"qps {qps}: {k + 1}/{len(texts)} sent, {len(done)} done", file=sys.stderr, flush=True)
                    t_note = time.perf_counter()
            await asyncio.gather(*tasks)
            wall = time.perf_counter() - t_start
            l = np.asarray(lat) * 1e3
            audio_s = sum(n for _, n in done) / 2 / 32000
            out.append({"offered_qps": qps, "requests": len(texts), "achieved_utt_s": len(texts) / wall,
                        "first_audio_ms_p50": float(np.percentile(l, 50)),
                        "first_audio_ms_p90": float(np.percentile(l, 90)),
                        "first_audio_ms_p99": float(np.percentile(l, 99)),
                        "total_ms_p50": float(np.percentile([d * 1e3 for d, _ in done], 50)),
                        "audio_s_per_wall_s": audio_s / wall})
            print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    server.should_exit = True
    await srv
    router.close()
    print(json.dumps({"workload": "configs[4]: FastAPI router + engine worker per GPU, Poisson QPS sweep, "
                                  "1 sentence (80 tokens, 3.2 s audio) per request",
                      "gpus": a.gpus, "startup_s": startup_s, "sweep": out}), flush=True)


if __name__ == "__main__":
    asyncio.run(main())
