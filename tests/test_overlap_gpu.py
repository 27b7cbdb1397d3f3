"""GPU: the overlapped vocoder (option "vocoder_cus", gsv_vits_decode_async /
gsv_vits_wait) -- a stream of sentences where sentence i's vocoder runs on its
own CUs beside sentence i+1's T2S (the reference runs them one after the other,
TTSPlayer._tts_worker_loop, Core/TTSPlayer.py:56-107).

Bars: with the decode on (256 - K) / 32 layer groups, every token bit-exact
against the reference-graph fixtures; every waveform RMS <= 1e-4 against them
(north_star) and identical to the engine's own sequential vocoder output; no
persistent-decode timeout (the CU split keeps the decode grid resident)."""
import os

import numpy as np
import pytest

from genie_tts_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.fixture(scope="module")
def eng():
    from genie_tts_amd.engine import Engine
    w = synth.synthetic_character("v2")
    e = Engine({k: w[k] for k in w}, "v2", pe_div_term=np.load(os.path.join(GOLD, "pe_div_term.npy")))
    e.set_option("persist", 1)
    yield e
    e.close()


@pytest.mark.parametrize("K", [64, 96, 32])
def test_overlapped_stream_matches_reference_graphs(eng, K):
    import torch
    from genie_tts_amd.engine import make_sampler
    t, nom, v = gold("t2s_nominal81.npz"), gold("t2s_nominal.npz"), gold("vits_v2_g80.npz")
    n = len(t["step_tokens"])
    smp = make_sampler(force_steps=n)
    utt = (nom["ref_seq"], nom["text_seq"], None, None, nom["ssl"])
    eng.set_vocoder_cus(0)
    seq_audio = eng.vits_decode(v["text_seq"], v["pred_semantic"], ref_audio=v["ref_audio"],
                                noise_seed=int(v["noise_seed"])).cpu()
    t0 = eng.counter("persist_timeouts")
    eng.set_vocoder_cus(K)
    try:
        audios = []
        for i in range(3):   # T2S of sentence i beside the vocoder of sentence i-1
            out = eng.t2s_generate([utt], smp)
            np.testing.assert_array_equal(out[0], t["pred_semantic"].reshape(-1))
            if i:
                eng.vits_wait()
            audios.append(eng.vits_decode_async(dict(text_seq=v["text_seq"], pred_semantic=v["pred_semantic"],
                                                     ref_audio=v["ref_audio"], noise_seed=int(v["noise_seed"]))))
        eng.vits_wait()
        for a in audios:
            a = a.cpu()
            assert torch.equal(a, seq_audio)
            rms = float(np.sqrt(np.mean((a.numpy() - v["audio_philox"]) ** 2)))
            assert rms <= 1e-4, rms
        assert eng.counter("persist_timeouts") == t0
    finally:
        eng.set_vocoder_cus(0)


def test_overlapped_vocoder_needs_the_split(eng):
    from genie_tts_amd.engine import EngineError
    v = gold("vits_v2_g80.npz")
    eng.set_vocoder_cus(0)
    with pytest.raises(EngineError, match="vocoder_cus"):
        eng.vits_decode_async(dict(text_seq=v["text_seq"], pred_semantic=v["pred_semantic"], ref_audio=v["ref_audio"]))
    for bad in (12, 4, 256, 200):
        with pytest.raises(EngineError, match="vocoder_cus"):
            eng.set_vocoder_cus(bad)
    eng.vits_wait()   # nothing pending: a no-op


def test_sync_vocoder_finishes_a_pending_call(eng):
    """A synchronous vocoder call after an async one: the pending call is finished
    first (they share the workspace), and both outputs are correct."""
    v = gold("vits_v2_g80.npz")
    kw = dict(ref_audio=v["ref_audio"])
    eng.set_vocoder_cus(64)
    try:
        a = eng.vits_decode_async(dict(text_seq=v["text_seq"], pred_semantic=v["pred_semantic"], **kw))
        b = eng.vits_decode(v["text_seq"], v["pred_semantic"], **kw)
        for x in (a, b):
            rms = float(np.sqrt(np.mean((x.cpu().numpy() - v["audio_zero"]) ** 2)))
            assert rms <= 1e-4, rms
    finally:
        eng.set_vocoder_cus(0)


@pytest.mark.parametrize("greedy", [True, False])
def test_prefetch_stream_matches_plain_generate(eng, greedy):
    """gsv_t2s_prefetch: sentence i+1 encoded and prefilled into slot 1 on the
    vocoder CUs while sentence i decodes, then taken into slot 0 -- every token
    identical to a plain generate of the same sentence, greedy and top-k sampled
    (the prefill draws slot 0's Philox noise), with BERT features and ragged
    lengths (the slot copy moves exactly the prefilled rows)."""
    from tests.common import t2s_inputs
    from genie_tts_amd.engine import make_sampler
    sp = make_sampler(top_k=15, greedy=greedy, seed=77, force_steps=24)
    utts = [t2s_inputs(R=10 + 3 * i, S=8 + 5 * i, H=30 + 12 * i, tag=f"pf{i}", bert=i % 2 == 1) for i in range(4)]
    eng.set_vocoder_cus(0)
    plain = [eng.t2s_generate([u], sp)[0] for u in utts]
    plain_batch = eng.t2s_generate(utts[:2], sp)
    t0 = eng.counter("persist_timeouts")
    eng.set_vocoder_cus(64)
    try:
        dev = [tuple(eng._dev(a, None) if a is not None else None for a in u) for u in utts]
        got = []
        for i in range(len(dev)):
            if i + 1 < len(dev):
                eng.t2s_prefetch(dev[i + 1], sp)
            got.append(eng.t2s_generate([dev[i]], sp)[0])
        for i, (a, b) in enumerate(zip(got, plain)):
            assert a.tolist() == b.tolist(), f"utterance {i}"
        assert eng.counter("persist_timeouts") == t0
        # a different utterance than the one prefetched: the plain path, still exact
        eng.t2s_prefetch(dev[1], sp)
        assert eng.t2s_generate([dev[2]], sp)[0].tolist() == plain[2].tolist()
        assert eng.t2s_generate([dev[3]], sp)[0].tolist() == plain[3].tolist()
        # a batch after a queued prefetch discards it
        eng.t2s_prefetch(dev[0], sp)
        out = eng.t2s_generate([dev[0], dev[1]], sp)
        assert [o.tolist() for o in out] == [o.tolist() for o in plain_batch]
    finally:
        eng.set_vocoder_cus(0)


def test_prefetch_needs_the_split(eng):
    from tests.common import t2s_inputs
    from genie_tts_amd.engine import EngineError
    eng.set_vocoder_cus(0)
    with pytest.raises(EngineError, match="vocoder_cus"):
        eng.t2s_prefetch(t2s_inputs(tag="pfx"))


@pytest.mark.parametrize("greedy", [True, False])
def test_async_generate_stream_matches_plain(eng, greedy):
    """gsv_t2s_generate_start / _finish with two in flight (utterance i+1 queued behind
    utterance i) and prefetches: every token identical to a plain generate."""
    from tests.common import t2s_inputs
    from genie_tts_amd.engine import make_sampler
    sp = make_sampler(top_k=15, greedy=greedy, seed=91, force_steps=20)
    utts = [t2s_inputs(R=11 + 2 * i, S=9 + 4 * i, H=33 + 10 * i, tag=f"as{i}", bert=i % 2 == 0) for i in range(5)]
    eng.set_vocoder_cus(0)
    plain = [eng.t2s_generate([u], sp)[0] for u in utts]
    eng.set_vocoder_cus(64)
    try:
        dev = [tuple(eng._dev(a, None) if a is not None else None for a in u) for u in utts]
        eng.t2s_prefetch(dev[1], sp)
        eng.t2s_generate_start(dev[0], sp)
        got = []
        for i in range(len(dev)):
            if i + 1 < len(dev):
                if i + 2 < len(dev):
                    eng.t2s_prefetch(dev[i + 2], sp)
                eng.t2s_generate_start(dev[i + 1], sp)
            got.append(eng.t2s_generate_finish())
        for i, (a, b) in enumerate(zip(got, plain)):
            assert a.tolist() == b.tolist(), f"utterance {i}"
        # no prefetch at all: the starts prefill themselves, still exact
        eng.t2s_generate_start(dev[3], sp)
        eng.t2s_generate_start(dev[4], sp)
        assert eng.t2s_generate_finish().tolist() == plain[3].tolist()
        # a synchronous generate in between waits for the started one; its result stays queued
        assert eng.t2s_generate([dev[2]], sp)[0].tolist() == plain[2].tolist()
        assert eng.t2s_generate_finish().tolist() == plain[4].tolist()
    finally:
        eng.set_vocoder_cus(0)


def test_async_generate_fp16_guard_reruns(eng):
    """A started generate whose persistent launch meets the (test-lowered) fp16 limit is
    re-run synchronously inside _finish: same tokens as the plain path."""
    from tests.common import t2s_inputs
    from genie_tts_amd.engine import make_sampler, EngineError
    sp = make_sampler(force_steps=12)
    u = t2s_inputs(R=12, S=10, H=41, tag="asf")
    ref = eng.t2s_generate([u], sp)[0]
    n0 = eng.counter("persist1_f16_reruns")
    eng.set_option("persist1_f16_limit", 1)
    try:
        eng.t2s_generate_start(u, sp)
        assert eng.t2s_generate_finish().tolist() == ref.tolist()
    finally:
        eng.set_option("persist1_f16_limit", 0)
    assert eng.counter("persist1_f16_reruns") > n0
    with pytest.raises(EngineError, match="no generate in flight"):
        eng.t2s_generate_finish()


@pytest.mark.parametrize("D,off", [(96, 0), (96, 96), (128, 32)])
def test_decode_cu_range(eng, D, off):
    """Options decode_cus / decode_cu_offset (several sentence streams sharing one GPU,
    bench.py --streams-per-gpu): the persistent decode on D CUs at an offset past the
    vocoder CUs gives the golden tokens, with no residency timeout."""
    from genie_tts_amd.engine import EngineError, make_sampler
    t, nom, v = gold("t2s_nominal81.npz"), gold("t2s_nominal.npz"), gold("vits_v2_g80.npz")
    smp = make_sampler(force_steps=len(t["step_tokens"]))
    utt = (nom["ref_seq"], nom["text_seq"], None, None, nom["ssl"])
    eng.set_vocoder_cus(0)
    t0 = eng.counter("persist_timeouts")
    try:
        eng.set_option("decode_cus", D)
        eng.set_option("decode_cu_offset", off)
        eng.set_vocoder_cus(64)
        for i in range(2):
            out = eng.t2s_generate([utt], smp)
            np.testing.assert_array_equal(out[0], t["pred_semantic"].reshape(-1))
            if i:
                eng.vits_wait()
            eng.vits_decode_async(dict(text_seq=v["text_seq"], pred_semantic=v["pred_semantic"],
                                       ref_audio=v["ref_audio"], noise_seed=int(v["noise_seed"])))
        eng.vits_wait()
        assert eng.counter("persist_timeouts") == t0
        for bad in (("decode_cus", 80), ("decode_cus", 224), ("decode_cu_offset", 4), ("decode_cu_offset", 160)):
            with pytest.raises(EngineError, match="decode_cu"):
                eng.set_option(*bad)
    finally:
        eng.set_vocoder_cus(0)
        eng.set_option("decode_cus", 0)
        eng.set_option("decode_cu_offset", 0)
