"""GPU: the persistent decode launches (t2s_persist1.hip at B = 1, its multi-sequence
form at B = 2..64) against the per-step hipGraph path (t2s_decode.hip), each other and
the CPU oracle.

Both decode paths sit behind gsv_t2s_generate (the reference's 500-step loop,
Inference.py:95-109); option "persist" selects one.  Bars: greedy token ids
identical to the oracle (bit-exact, north_star) and to the graph path; sampled
(top-k, Philox) ids identical to the graph path -- same sampler formula and
noise, only the block size of the sampler's reductions differs.
"""
import numpy as np
import pytest

from tests.common import character, t2s_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from genie_tts_amd.engine import Engine
    w = character("v2")
    e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
    yield e
    e.close()


@pytest.fixture(scope="module")
def oracle_model():
    from oracle import restate as R
    return R.T2SModel(character("v2")["t2s"])


def _both(eng, inps, sp):
    eng.set_option("persist", 1)
    a = eng.t2s_generate(inps, sp)
    eng.set_option("persist", 0)
    try:
        b = eng.t2s_generate(inps, sp)
    finally:
        eng.set_option("persist", 1)
    return a, b


def _ordered(inp):
    ref, txt, rb, tb, ssl = inp
    return ref, rb, txt, tb, ssl


@pytest.mark.parametrize("R_,S_,H_,steps", [(12, 10, 41, 30), (48, 45, 264, 81)])
def test_persistent_greedy_matches_oracle(eng, oracle_model, R_, S_, H_, steps):
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inp = t2s_inputs(R=R_, S=S_, H=H_, tag=f"p{R_}")
    eng.set_option("persist", 1)
    out = eng.t2s_generate([inp], make_sampler(force_steps=steps))
    sem, _, _ = R.t2s_generate(character("v2")["t2s_encoder"], oracle_model, *_ordered(inp), force_steps=steps)
    assert out[0].tolist() == sem.reshape(-1).tolist()


def test_persistent_long_context_multipass(eng, oracle_model):
    """N0 = 93 + 300 > 384 keys: attention runs past the LDS-staged rows."""
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inp = t2s_inputs(R=48, S=45, H=600, tag="long")
    steps = 12
    eng.set_option("persist", 1)
    out = eng.t2s_generate([inp], make_sampler(force_steps=steps))
    sem, _, _ = R.t2s_generate(character("v2")["t2s_encoder"], oracle_model, *_ordered(inp), force_steps=steps)
    assert out[0].tolist() == sem.reshape(-1).tolist()


@pytest.mark.parametrize("B", [1, 3, 8])
def test_persistent_matches_graph_path_greedy(eng, B):
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + 2 * i, S=8 + i, H=30 + 4 * i, tag=f"pg{B}_{i}") for i in range(B)]
    a, b = _both(eng, inps, make_sampler(force_steps=20))
    for i in range(B):
        assert a[i].tolist() == b[i].tolist(), f"utterance {i}"


@pytest.mark.parametrize("top_k,temp", [(15, 1.0), (5, 0.8)])
def test_persistent_matches_graph_path_sampled(eng, top_k, temp):
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=12 + i, S=9 + i, H=36 + 2 * i, tag=f"ps{i}") for i in range(4)]
    sp = make_sampler(top_k=top_k, temperature=temp, greedy=False, seed=1234, force_steps=24)
    a, b = _both(eng, inps, sp)
    for i in range(len(inps)):
        assert a[i].tolist() == b[i].tolist(), f"utterance {i}"


def test_persistent_natural_stop_max_steps(eng):
    """No forced length: the loop ends on max_steps (Inference.py:95 range(500)) -> idx+1 tokens."""
    from genie_tts_amd.engine import make_sampler
    inp = t2s_inputs(R=10, S=8, H=30, tag="ms")
    a, b = _both(eng, [inp], make_sampler(max_steps=17))
    assert a[0].tolist() == b[0].tolist()
    assert len(a[0]) > 0


@pytest.mark.parametrize("B", [1, 4])
def test_persistent_full_500_step_loop(eng, B):
    """The reference's whole loop (Inference.py:95, range(500)) with no EOS (random
    weights): 500 steps, the keys growing past the LDS stage (N0 ~ 150 + 500 > 448
    rows) -- the persistent kernels equal the per-step graphs at the maximum length."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=40 + 3 * i, S=30 + 2 * i, H=160 + 8 * i, tag=f"f500_{B}_{i}") for i in range(B)]
    a, b = _both(eng, inps, make_sampler())
    for i in range(B):
        assert a[i].tolist() == b[i].tolist(), f"utterance {i}"
        assert len(a[i]) >= 450       # no EOS under random weights: (nearly) the whole loop


def test_persistent_fp16_range_fallback(eng, oracle_model):
    """An FFN activation beyond the fp16 range of the single-sequence kernel's split
    MFMA operands stops it (error code 2) and the host re-runs the steps as per-step
    graphs.  The hook lowers the limit to 1.0 so that the fallback fires; the tokens
    stay bit-exact vs the oracle."""
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inp = t2s_inputs(R=12, S=10, H=41, tag="p12")
    steps = 30
    eng.set_option("persist", 1)
    eng.set_option("persist1_f16_limit", 1)
    try:
        out = eng.t2s_generate([inp], make_sampler(force_steps=steps))
    finally:
        eng.set_option("persist1_f16_limit", 0)
    sem, _, _ = R.t2s_generate(character("v2")["t2s_encoder"], oracle_model, *_ordered(inp), force_steps=steps)
    assert out[0].tolist() == sem.reshape(-1).tolist()


def test_persistent_repeated_calls_are_deterministic(eng):
    from genie_tts_amd.engine import make_sampler
    inp = t2s_inputs(R=14, S=11, H=44, tag="rep")
    sp = make_sampler(top_k=15, greedy=False, seed=7, force_steps=30)
    eng.set_option("persist", 1)
    first = eng.t2s_generate([inp], sp)[0].tolist()
    for _ in range(3):
        assert eng.t2s_generate([inp], sp)[0].tolist() == first


def test_persistent_timeout_reruns_as_graphs(eng):
    """A hand-off that waits past its bound (co-running work on the device) makes the
    persistent launch leave without writing the sequence state; the same steps then
    run as per-step graphs and the tokens stay bit-exact (forced here with a 0.5 us
    bound)."""
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inp = t2s_inputs(R=12, S=10, H=41, tag="tmo")
    before = eng.counter("persist_timeouts")
    eng.set_option("persist_spin_ticks", 50)
    try:
        out = eng.t2s_generate([inp], make_sampler(force_steps=12))
    finally:
        eng.set_option("persist_spin_ticks", 0)
    assert eng.counter("persist_timeouts") > before
    ref, txt, rb, tb, ssl = inp
    sem, _, _ = R.t2s_generate(character("v2")["t2s_encoder"], R.T2SModel(character("v2")["t2s"]), ref, rb, txt,
                               tb, ssl, force_steps=12)
    assert out[0].tolist() == sem.reshape(-1).tolist()


def test_repeated_timeouts_leave_the_persistent_path(eng):
    """Two timed-out launches in a row (the grid cannot be co-resident) start a back-off hold
    on the per-step graphs, so the next utterances do not pay the wait bound; option
    persist = 1 ends the hold."""
    from genie_tts_amd.engine import make_sampler
    inp = t2s_inputs(R=12, S=10, H=41, tag="tmo2")
    sp = make_sampler(force_steps=10)
    eng.set_option("persist", 1)
    want = eng.t2s_generate([inp], sp)[0].tolist()
    before = eng.counter("persist_timeouts")
    eng.set_option("persist_spin_ticks", 50)
    try:
        for _ in range(3):
            assert eng.t2s_generate([inp], sp)[0].tolist() == want
    finally:
        eng.set_option("persist_spin_ticks", 0)
    assert eng.counter("persist_timeouts") == before + 2     # the third ran on the graphs directly
    eng.set_option("persist", 1)
    assert eng.t2s_generate([inp], sp)[0].tolist() == want
    assert eng.counter("persist_timeouts") == before + 2


def _alone(eng, inps, sp):
    return [eng.t2s_generate([inp], sp)[0].tolist() for inp in inps]


@pytest.mark.parametrize("B", [2, 5, 8, 16, 40, 64])
def test_multi_sequence_matches_single_launches(eng, B):
    """The multi-sequence form of the single-sequence kernel (k_decode_persist1m, B = 2..64)
    runs every sequence through the same per-sequence arithmetic: each sequence's greedy
    tokens are the ones a launch of its own gives (k_decode_persist1)."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"m{B}_{i}") for i in range(B)]
    sp = make_sampler(force_steps=22)
    eng.set_option("persist", 1)
    got = eng.t2s_generate(inps, sp)
    assert [g.tolist() for g in got] == _alone(eng, inps, sp)


def test_multi_sequence_ragged_lengths(eng):
    """Sequences that finish at different steps (per-utterance forced lengths) leave the
    launch one by one; the others keep their tokens (vs the per-step graph path and vs
    launches of their own)."""
    from genie_tts_amd.engine import make_sampler
    lens = [9, 25, 4, 17, 12]
    inps = [t2s_inputs(R=11 + i, S=9 + i, H=32 + 4 * i, tag=f"rg{i}") + (n,) for i, n in enumerate(lens)]
    sp = make_sampler(force_steps=30)
    a, b = _both(eng, inps, sp)
    for i in range(len(lens)):
        assert a[i].tolist() == b[i].tolist(), f"utterance {i}"
    assert len({len(x) for x in a}) == len(lens)   # every sequence stopped at its own step
    assert [x.tolist() for x in a] == _alone(eng, inps, sp)


def test_multi_sequence_fp16_range_fallback(eng):
    """An activation past the fp16 range stops the multi-sequence launch (error 2) before
    any sequence state is written; the steps run again as per-step graphs with the
    same tokens."""
    from genie_tts_amd.engine import make_sampler
    for B in (3, 12):
        inps = [t2s_inputs(R=10 + i, S=8 + i, H=30 + 2 * i, tag=f"mf{B}_{i}") for i in range(B)]
        sp = make_sampler(force_steps=14)
        eng.set_option("persist", 1)
        ref = eng.t2s_generate(inps, sp)
        before = eng.counter("persist1_f16_reruns")
        eng.set_option("persist1_f16_limit", 1)
        try:
            got = eng.t2s_generate(inps, sp)
        finally:
            eng.set_option("persist1_f16_limit", 0)
        assert eng.counter("persist1_f16_reruns") > before
        assert [g.tolist() for g in got] == [r.tolist() for r in ref]


def test_multi_sequence_sampled_matches_graph_path(eng):
    """Top-k sampling at B = 3: the multi-sequence kernel's sampler workgroups (one per
    sequence) draw what the per-step graphs' sampler draws (same Philox keys; option
    persist1m = 0 sends B > 1 to the graphs)."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=12 + i, S=9 + i, H=36 + 2 * i, tag=f"msk{i}") for i in range(3)]
    sp = make_sampler(top_k=15, greedy=False, seed=99, force_steps=20)
    eng.set_option("persist", 1)
    a = eng.t2s_generate(inps, sp)
    eng.set_option("persist1m", 0)
    try:
        b = eng.t2s_generate(inps, sp)
    finally:
        eng.set_option("persist1m", 1)
    for i in range(len(inps)):
        assert a[i].tolist() == b[i].tolist(), f"utterance {i}"


def test_timeout_backoff_reprobes_the_persistent_path(eng):
    """After two timeouts in a row the engine holds on the per-step graphs for a bounded
    number of generates (option persist_backoff), then probes the persistent path again:
    once the condition has cleared, it is back (persist_launches grows again); tokens are
    bit-exact throughout.  A probe that times out again starts a longer hold."""
    from genie_tts_amd.engine import make_sampler
    inp = t2s_inputs(R=12, S=10, H=41, tag="bko")
    sp = make_sampler(force_steps=10)
    eng.set_option("persist", 1)
    eng.set_option("persist_backoff", 3)
    eng.set_option("persist_backoff_ms", 600000)
    try:
        want = eng.t2s_generate([inp], sp)[0].tolist()
        t0, d0 = eng.counter("persist_timeouts"), eng.counter("persist_disabled")
        eng.set_option("persist_spin_ticks", 50)
        try:
            for _ in range(2):
                assert eng.t2s_generate([inp], sp)[0].tolist() == want
        finally:
            eng.set_option("persist_spin_ticks", 0)
        assert eng.counter("persist_timeouts") == t0 + 2
        assert eng.counter("persist_disabled") == d0 + 1 and eng.counter("persist_hold") == 3
        n0 = eng.counter("persist_launches")
        for _ in range(2):                       # the hold: per-step graphs, no launch
            assert eng.t2s_generate([inp], sp)[0].tolist() == want
        assert eng.counter("persist_launches") == n0
        for k in (1, 2):                         # the probe succeeds; the path stays
            assert eng.t2s_generate([inp], sp)[0].tolist() == want
            assert eng.counter("persist_launches") == n0 + k
        assert eng.counter("persist_timeouts") == t0 + 2 and eng.counter("persist_hold") == 0
        # the condition returns: two timeouts -> a hold of 3 (the successful launches reset
        # the back-off); its probe times out again -> a hold twice as long
        eng.set_option("persist_spin_ticks", 50)
        try:
            for _ in range(2):
                assert eng.t2s_generate([inp], sp)[0].tolist() == want
            assert eng.counter("persist_hold") == 3
            for _ in range(3):                   # 2 on the graphs, then the failing probe
                assert eng.t2s_generate([inp], sp)[0].tolist() == want
        finally:
            eng.set_option("persist_spin_ticks", 0)
        assert eng.counter("persist_timeouts") == t0 + 5
        assert eng.counter("persist_hold") == 6
    finally:
        eng.set_option("persist_backoff", 64)
        eng.set_option("persist_backoff_ms", 5000)
        eng.set_option("persist", 1)


def _stop_during(eng, inps, sp, persist, delay_s):
    """Request a stop `delay_s` into a generate; returns (raised EngineStopped, seconds from
    the request to the generate's return, seconds the generate ran)."""
    import threading
    import time
    from genie_tts_amd.engine import EngineStopped
    eng.set_option("persist", persist)
    res = {}

    def run():
        t = time.perf_counter()
        try:
            eng.t2s_generate(inps, sp)
            res["stopped"] = False
        except EngineStopped:
            res["stopped"] = True
        res["end"] = time.perf_counter()
        res["ran"] = res["end"] - t
    th = threading.Thread(target=run)
    th.start()
    time.sleep(delay_s)
    t_req = time.perf_counter()
    eng.request_stop(True)
    th.join(timeout=30)
    assert not th.is_alive()
    eng.request_stop(False)
    eng.set_option("persist", 1)
    return res["stopped"], res["end"] - t_req, res["ran"]


@pytest.mark.parametrize("B,persist", [(1, 1), (8, 1), (1, 0)])
def test_stop_interrupts_a_running_decode(eng, B, persist):
    """gsv_request_stop during a forced 500-step decode (the reference's stop_event,
    checked every loop step, Inference.py:96-97): the generate raises EngineStopped within
    a few steps of the request (a step is ~0.2 ms at B = 1), the stop counter grows, and
    the engine decodes the same utterances bit-exactly afterwards."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=12 + i, S=10 + i, H=41, tag=f"stp{i}") for i in range(B)]
    sp = make_sampler(force_steps=500)
    eng.set_option("persist", 1)
    full = eng.t2s_generate(inps, sp)                 # warm, and the uninterrupted tokens
    import time
    t = time.perf_counter()
    eng.t2s_generate(inps, sp)
    t_full = time.perf_counter() - t
    s0 = eng.counter("stops")
    stopped, latency, ran = _stop_during(eng, inps, sp, persist, 0.3 * t_full)
    print(f"B={B} persist={persist}: full {t_full * 1e3:.1f} ms, stopped after {ran * 1e3:.1f} ms, "
          f"{latency * 1e3:.2f} ms after the request")
    assert stopped and eng.counter("stops") == s0 + 1
    assert ran < 0.8 * t_full
    # two loop steps of this decode plus the host's wake-up; the graph path checks its
    # stop word per step too, but its host loop keeps two 8-step chunks queued ahead and
    # notices only between them (measured r04l: 4.08 ms at 0.2 ms per step)
    step = t_full / 500
    assert latency < 2 * step + (16 * step if persist == 0 else 0) + 2e-3, latency
    # a request before the call: nothing runs
    eng.request_stop(True)
    from genie_tts_amd.engine import EngineStopped
    with pytest.raises(EngineStopped):
        eng.t2s_generate(inps, sp)
    eng.request_stop(False)
    again = eng.t2s_generate(inps, sp)
    assert [a.tolist() for a in again] == [f.tolist() for f in full]
