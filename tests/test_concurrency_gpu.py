"""GPU: the engine under concurrent issue (gpurun_out/r04o_probe.err).

- One engine: a per-step-graph generate (persist 0) whose graph key is new -- so its
  decode loop captures hipGraphs -- issued while a gsv_vits_decode_batch_async batch that
  grows the lanes' workspaces is in flight.  Tokens equal the same generate run alone, the
  audio equals the synchronous batch call bit for bit, no GSV_E_HIP.
- Several engines in one process, one host thread each, all capturing step graphs at once
  (the r04o probe that failed with "decode graph capture failed" / "encode launch"): every
  thread's tokens equal the sequential run.
A capture that another thread's device-wide synchronisation invalidates falls back to
eager launches of the same kernels (counter graph_fallbacks), so results never depend on it.
Reference loop: Core/TTSPlayer.py:55-114 (one sentence after another per worker).
"""
import threading

import numpy as np
import pytest

from genie_tts_amd import synth, workloads
from tests.common import character

pytestmark = pytest.mark.gpu


def _utt(torch, force_steps=40):
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    T = lambda a: torch.as_tensor(a, device="cuda")
    return (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
            force_steps)


def _items(n, G0, tag):
    ref_audio = synth.synth_ref_audio(32000 * 2 + 777)
    out = []
    for i in range(n):
        G = G0 + 7 * i
        txt = synth.synth_phones(10 + 3 * i, f"{tag}t{i}")
        sem = ((np.arange(G, dtype=np.int64) * (3 + i) + 11 * i) % 1024).reshape(1, 1, G)
        out.append(dict(text_seq=txt, pred_semantic=sem, ref_audio=ref_audio, noise_seed=500 + i))
    return out


def test_graph_capture_beside_growing_vocoder_batch():
    import torch
    from genie_tts_amd.engine import Engine, make_sampler
    e = Engine({k: v for k, v in character("v2").items() if k in ("t2s_encoder", "t2s", "vits")}, "v2")
    try:
        utt = _utt(torch)
        e.vits_decode_batch(_items(4, 12, "warm"))           # lanes exist, small workspaces
        e.set_option("persist", 0)
        sp = make_sampler(greedy=False, top_k=7, seed=4242)  # a sampler no graph was captured for
        big = _items(6, 60, "big")                           # longer than anything before: workspaces grow
        for seg in (1, 0):
            e.set_option("seg_vocoder", seg)
            outs = e.vits_decode_batch_async(big)
            toks_c = e.t2s_generate([utt] * 3, sp)
            e.vits_batch_wait()
            audio_c = [o.cpu().numpy() for o in outs]
            toks_s = e.t2s_generate([utt] * 3, sp)
            audio_s = [o.cpu().numpy() for o in e.vits_decode_batch(big)]
            for a, b in zip(toks_c, toks_s):
                np.testing.assert_array_equal(a, b)
            for i, (a, b) in enumerate(zip(audio_c, audio_s)):
                np.testing.assert_array_equal(a, b, err_msg=f"seg {seg} item {i}")
            sp = make_sampler(greedy=False, top_k=9, seed=4243)   # a new key for the next round too
    finally:
        e.set_option("seg_vocoder", 1)
        e.set_option("persist", 1)
        e.close()


def test_engines_capturing_on_concurrent_threads():
    import torch
    from genie_tts_amd.engine import Engine, make_sampler
    ch = {k: v for k, v in character("v2").items() if k in ("t2s_encoder", "t2s")}
    engines = [Engine(ch, "v2") for _ in range(4)]
    try:
        utt = _utt(torch)
        streams = [torch.cuda.Stream() for _ in engines]
        for e in engines:
            e.set_option("persist1m", 0)      # B > 1 on the per-step graphs: every engine captures
        # B = 16: past the engines' initial capacity, so the threads' first generates grow their
        # state (reserve) while other engines capture -- the r04o failure (tools/concurrency_probe.py)
        ref = engines[0].t2s_generate([utt] * 16, make_sampler())
        res, errs = [None] * len(engines), []

        def work(i, sampler):
            try:
                with torch.cuda.stream(streams[i]):
                    res[i] = engines[i].t2s_generate([utt] * 16, sampler)
            except Exception as ex:   # collected: an error in a thread must fail the test
                errs.append(f"engine {i}: {ex}")

        for rnd in range(3):   # round 0: engine 0's key exists, the others capture; later rounds: new keys
            sp = make_sampler() if rnd == 0 else make_sampler(max_steps=400 + rnd)
            th = [threading.Thread(target=work, args=(i, sp)) for i in range(len(engines))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            torch.cuda.synchronize()
            assert not errs, errs
            for r in res:
                for a, b in zip(r, ref):
                    np.testing.assert_array_equal(a, b)
        # growth frees its retired buffers under the process-wide capture lock, so no thread's
        # device-synchronising free invalidates another's capture: no eager fallback was needed
        assert [e.counter("graph_fallbacks") for e in engines] == [0] * len(engines)
    finally:
        for e in engines:
            e.close()


def test_back_to_back_async_batches_on_the_f32_path():
    """Two gsv_vits_decode_batch_async batches in a row from a stream other than the engine
    stream, on the f32 conv path (convh = 0, no fp16-range host sync), segmented and per
    lane: the second batch's setup (offset tables, zeroed buffers) waits for the first
    batch's lanes, so each batch equals its synchronous call bit for bit."""
    import torch
    from genie_tts_amd.engine import Engine
    e = Engine({k: v for k, v in character("v2").items() if k in ("t2s_encoder", "t2s", "vits")}, "v2")
    try:
        e.set_option("convh", 0)
        first, second = _items(5, 30, "ba"), _items(4, 52, "bb")
        for seg in (1, 0):
            e.set_option("seg_vocoder", seg)
            want = [[o.cpu().numpy() for o in e.vits_decode_batch(b)] for b in (first, second)]
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                outs_a = e.vits_decode_batch_async(first)
                outs_b = e.vits_decode_batch_async(second)
                e.vits_batch_wait()
            st.synchronize()
            for k, (outs, w) in enumerate(zip((outs_a, outs_b), want)):
                for i, (o, x) in enumerate(zip(outs, w)):
                    np.testing.assert_array_equal(o.cpu().numpy(), x, err_msg=f"seg {seg} batch {k} item {i}")
    finally:
        e.set_option("seg_vocoder", 1)
        e.set_option("convh", 1)
        e.close()
