"""T2S parity on the GPU: the HIP engine through the C ABI vs the CPU oracle.

Oracle = oracle/restate.py (torch fp32), itself pinned to the reference graph
templates by tests/test_oracle.py and tests/golden/.  Tolerances: fp32
activations with different reduction orders -> 2e-4 abs on O(1) tensors;
greedy token ids must be identical (bit-exact, the north_star's bar).
"""
import numpy as np
import pytest
import torch

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


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("bert", [False, True])
def test_encoder(eng, bert):
    from oracle import restate as R
    ref, txt, rb, tb, ssl = t2s_inputs(R=12, S=10, H=41, tag="e", bert=bert)
    x, prompts = eng.t2s_encode(ref, txt, rb if bert else None, tb if bert else None, ssl)
    xr, pr = R.t2s_encoder(character("v2")["t2s_encoder"], ref, txt, rb, tb, ssl)
    np.testing.assert_array_equal(_np(prompts), pr.numpy().reshape(-1))
    np.testing.assert_allclose(_np(x), xr.numpy().reshape(-1, 512), atol=2e-5, rtol=1e-5)


def test_prefill_and_steps(eng, oracle_model):
    from oracle import restate as R
    ref, txt, rb, tb, ssl = t2s_inputs(R=12, S=10, H=41, tag="p")
    xr, pr = R.t2s_encoder(character("v2")["t2s_encoder"], ref, txt, rb, tb, ssl)
    y, logits = eng.t2s_prefill(xr.numpy().reshape(-1, 512), pr.numpy())
    st, lref = R.t2s_prefill(oracle_model, xr, pr.numpy(), torch.ones(1025))
    np.testing.assert_allclose(_np(logits), lref.numpy(), atol=2e-4, rtol=1e-4)
    assert _np(y).tolist() == st.y
    for layer in (0, 23):
        k, v = eng.t2s_read_kv(layer)
        np.testing.assert_allclose(_np(k), st.k[layer].numpy(), atol=2e-4, rtol=1e-4)
        np.testing.assert_allclose(_np(v), st.v[layer].numpy(), atol=2e-4, rtol=1e-4)
    steps = 6
    y2, stop, lg = eng.t2s_decode_steps(steps)
    for i in range(steps):
        s_ref, l_ref = R.t2s_step(oracle_model, st, torch.ones(1025))
        np.testing.assert_allclose(_np(lg[i]), l_ref.numpy(), atol=5e-4, rtol=1e-4)
        assert int(stop[i]) == int(s_ref)
    n = len(st.y)
    assert _np(y2[:n]).tolist() == st.y


@pytest.mark.parametrize("R_,S_,H_", [(12, 10, 41), (48, 45, 264)])
def test_generate_greedy_bitexact(eng, oracle_model, R_, S_, H_):
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inp = t2s_inputs(R=R_, S=S_, H=H_, tag=f"g{R_}")
    steps = 24 if R_ < 40 else 40
    out = eng.t2s_generate([inp], make_sampler(force_steps=steps))
    sem, st, _ = R.t2s_generate(character("v2")["t2s_encoder"], oracle_model, *_ordered(inp),
                                force_steps=steps)
    assert out[0].tolist() == sem.reshape(-1).tolist()


def _ordered(inp):
    ref, txt, rb, tb, ssl = inp
    return ref, rb, txt, tb, ssl


def test_generate_batch_matches_single(eng):
    from genie_tts_amd.engine import make_sampler
    inps = [t2s_inputs(R=12 + 3 * i, S=10 + 2 * i, H=41 + 6 * i, tag=f"b{i}") for i in range(3)]
    sp = make_sampler(force_steps=16)
    batch = eng.t2s_generate(inps, sp)
    for i, inp in enumerate(inps):
        single = eng.t2s_generate([inp], sp)
        assert batch[i].tolist() == single[0].tolist()


@pytest.mark.parametrize("B", [5, 10])
def test_generate_batched_paths_vs_oracle(eng, oracle_model, B):
    """B <= 8 runs the fused GEMV path, B > 8 the MFMA-GEMM path; both must
    reproduce the oracle's greedy tokens per utterance."""
    from genie_tts_amd.engine import make_sampler
    from oracle import restate as R
    inps = [t2s_inputs(R=8 + i, S=6 + (i % 3), H=20 + 2 * i, tag=f"bb{B}_{i}") for i in range(B)]
    out = eng.t2s_generate(inps, make_sampler(force_steps=12))
    for i, inp in enumerate(inps):
        sem, _, _ = R.t2s_generate(character("v2")["t2s_encoder"], oracle_model, *_ordered(inp),
                                   force_steps=12)
        assert out[i].tolist() == sem.reshape(-1).tolist(), f"utterance {i}"
