"""GPU: the batched persistent decode (k_decode_persistm, t2s_persistm.hip; the batch on
the MFMA M dimension, up to 4 sequences per group of 16 workgroups) against single
launches (k_decode_persist1) and the per-step graph path (t2s_decode.hip), both pinned to
the oracle by test_persist_gpu.py / test_golden_gpu.py.

Every sequence's values are the single-sequence kernel's (same K chains, folds and sum
orders; an MFMA output row depends on its own A row only), so greedy tokens are
bit-identical to a launch of its own; sampled tokens (Philox top-k) equal the graph
path's sampler.  Reference loop: Inference.py:95-106 (t2s_stage_decoder_fp32.onnx).

test_batched_generate_equals_single_at_a_near_tie pins the case found this round: a
batch's packed prefill on the split-fp16 MFMA attention flipped a near-tie token against
the sentence alone and the oracle; the packed prefill now runs the f32 kernels.
"""
import pytest

from tests.common import character, t2s_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from genie_tts_amd.engine import Engine
    w = character("v2")
    e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
    e.set_option("persist", 1)
    e.set_option("persistm", 1)
    e.set_option("persistm_min_b", 2)   # every B > 1 on the batched kernel unless persistm = 0
    yield e
    e.close()


def _both(eng, inps, sp):
    """persistm's tokens and the per-step graph path's"""
    n0 = eng.counter("persist_launches")
    a = [x.tolist() for x in eng.t2s_generate(inps, sp)]
    assert eng.counter("persist_launches") == n0 + 1   # one batched persistent launch
    eng.set_option("persist", 0)
    try:
        b = [x.tolist() for x in eng.t2s_generate(inps, sp)]
    finally:
        eng.set_option("persist", 1)
    return a, b


@pytest.mark.parametrize("B", [2, 4, 5, 17, 40, 64])
def test_batched_matches_graph_path(eng, B):
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm{B}_{i}") for i in range(B)]
    a, b = _both(eng, inps, make_sampler(force_steps=22))
    for i in range(B):
        assert a[i] == b[i], f"sequence {i}"


@pytest.mark.parametrize("B,tag", [(7, "pms"), (64, "pm64_")])
def test_batched_matches_single_launches(eng, B, tag):
    from genie_tts_amd.engine import make_sampler
    if B == 64:
        inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"{tag}{i}") for i in range(B)]
        sp = make_sampler(force_steps=22)
    else:
        inps = [t2s_inputs(R=12 + 5 * i, S=9 + 3 * i, H=40 + 9 * i, tag=f"{tag}{i}") for i in range(B)]
        sp = make_sampler(force_steps=30)
    got = [x.tolist() for x in eng.t2s_generate(inps, sp)]
    assert got == [eng.t2s_generate([inp], sp)[0].tolist() for inp in inps]


@pytest.mark.parametrize("persistm", [1, 0])
def test_batched_generate_equals_single_at_a_near_tie(eng, persistm):
    """Input 62 of the B = 64 set (730 prompt positions) sits at a near-tie at its second
    token: with the packed prefill's attention on the split-fp16 MFMA kernel (r04 default)
    a batched generate picked 217 where the sentence alone and the CPU oracle pick 444.
    Since r05 the packed prefill runs the f32 kernels the single prefill runs; both decode
    kernels (persistm, persist1m) then give the single launch's tokens."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm64_{i}") for i in (62, 0)]
    sp = make_sampler(force_steps=6)
    single = eng.t2s_generate([inps[0]], sp)[0].tolist()
    assert single[:2] == [842, 444]   # the oracle's (oracle/restate.py, CPU)
    eng.set_option("persistm", persistm)
    try:
        got = eng.t2s_generate(inps, sp)[0].tolist()
    finally:
        eng.set_option("persistm", 1)
    assert got == single


@pytest.mark.parametrize("top_k,temp", [(15, 1.0), (5, 0.8)])
def test_batched_sampled_matches_graph_path(eng, top_k, temp):
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=12 + i, S=9 + i, H=36 + 2 * i, tag=f"pmk{i}") for i in range(6)]
    a, b = _both(eng, inps, make_sampler(top_k=top_k, temperature=temp, greedy=False, seed=77, force_steps=24))
    for i in range(len(inps)):
        assert a[i] == b[i], f"sequence {i}"


def test_batched_ragged_lengths(eng):
    """Per-sequence forced lengths: sequences leave the launch one by one, the others keep
    their tokens; every sequence stops at its own step."""
    from genie_tts_amd.engine import make_sampler
    lens = [9, 25, 4, 17, 12, 30, 2, 21, 14]
    inps = [t2s_inputs(R=11 + i, S=9 + i, H=32 + 4 * i, tag=f"pmr{i}") + (n,) for i, n in enumerate(lens)]
    a, b = _both(eng, inps, make_sampler(force_steps=30))
    assert a == b
    assert [len(x) for x in a] == [len(x) for x in b]
    assert len({len(x) for x in a}) == len(set(lens))


def test_batched_long_context(eng):
    """Keys past the 448-row LDS stage (the general attention path) and past 512 keys."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=40 + 10 * i, S=30 + 5 * i, H=400 + 60 * i, tag=f"pml{i}") for i in range(5)]
    a, b = _both(eng, inps, make_sampler(force_steps=40))
    assert a == b


def test_batched_fp16_range_fallback(eng):
    """An activation past the fp16 range stops the batched launch (error 2) before any
    sequence state is written; the steps re-run as per-step graphs with the same tokens."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + i, S=8 + i, H=30 + 2 * i, tag=f"pmf{i}") for i in range(9)]
    sp = make_sampler(force_steps=14)
    ref = eng.t2s_generate(inps, sp)
    before = eng.counter("persist1_f16_reruns")
    eng.set_option("persist1_f16_limit", 1)
    try:
        got = eng.t2s_generate(inps, sp)
    finally:
        eng.set_option("persist1_f16_limit", 0)
    assert eng.counter("persist1_f16_reruns") > before
    assert [g.tolist() for g in got] == [r.tolist() for r in ref]


def test_batched_full_500_step_loop(eng):
    """The reference's whole loop (Inference.py:95, range(500)) with no EOS (random
    weights): keys grow past the LDS stage; tokens equal the graph path's at the maximum length."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=40 + 3 * i, S=30 + 2 * i, H=160 + 8 * i, tag=f"pm500_{i}") for i in range(6)]
    a, b = _both(eng, inps, make_sampler())
    assert a == b
    assert all(len(x) >= 450 for x in a)


def test_batched_stop_interrupts_and_writes_no_state(eng):
    """gsv_request_stop during a forced 500-step batched decode at B = 32 (the default path
    from persistm_min_b = 32; the reference's stop_event, Inference.py:96-97): the launch
    reads the stop word every 4th step and leaves with error 3 before the sequence-state
    write-back, so every sequence's KV length is still its prefill length; the generate
    raises EngineStopped well before the full run, and the same batch decodes bit-exactly
    afterwards (ADVICE r05 test_persistm_gpu.py:22)."""
    import time
    from genie_tts_amd.engine import make_sampler
    from tests.test_persist_gpu import _stop_during
    B = 32
    inps = [t2s_inputs(R=10 + i % 7, S=8 + i % 5, H=30 + 2 * i, tag=f"pmst{i}") for i in range(B)]
    sp = make_sampler(force_steps=500)
    full = eng.t2s_generate(inps, sp)
    t = time.perf_counter()
    eng.t2s_generate(inps, sp)
    t_full = time.perf_counter() - t
    s0, l0 = eng.counter("stops"), eng.counter("persist_launches")
    stopped, latency, ran = _stop_during(eng, inps, sp, 1, 0.3 * t_full)
    print(f"B={B}: full {t_full * 1e3:.1f} ms, stopped after {ran * 1e3:.1f} ms, {latency * 1e3:.2f} ms after the request")
    assert stopped and eng.counter("stops") == s0 + 1
    assert eng.counter("persist_launches") == l0 + 1   # it was the batched persistent launch
    assert ran < 0.8 * t_full
    step = t_full / 500
    assert latency < 6 * step + 2e-3, latency          # <= 4 steps to the next stop read, plus the exit
    for b in (0, 13, 31):                              # no sequence state written back
        k, _ = eng.t2s_read_kv(0, seq=b)
        R_, S_, H_ = 10 + b % 7, 8 + b % 5, 30 + 2 * b
        assert k.shape[0] == R_ + S_ + H_ // 2, (b, k.shape)
    again = eng.t2s_generate(inps, sp)
    assert [a.tolist() for a in again] == [f.tolist() for f in full]


def test_batched_timeout_reruns_as_graphs(eng):
    """A hand-off that waits past its bound (forced with a 0.5 us bound) makes the batched
    launch leave without writing the sequence state (error 1); the steps re-run on the
    per-step graphs and every sequence's tokens equal the graph path's."""
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=10 + i, S=8 + i, H=30 + 3 * i, tag=f"pmto{i}") for i in range(9)]
    sp = make_sampler(force_steps=16)
    eng.set_option("persist", 0)
    try:
        want = [x.tolist() for x in eng.t2s_generate(inps, sp)]
    finally:
        eng.set_option("persist", 1)
    before = eng.counter("persist_timeouts")
    eng.set_option("persist_spin_ticks", 50)
    try:
        got = [x.tolist() for x in eng.t2s_generate(inps, sp)]
    finally:
        eng.set_option("persist_spin_ticks", 0)
        eng.set_option("persist", 1)   # ends a back-off hold the timeout may have started
    assert eng.counter("persist_timeouts") == before + 1
    assert got == want
