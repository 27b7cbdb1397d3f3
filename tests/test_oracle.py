"""CPU: the oracle restatement (oracle/restate.py) against the golden fixtures
produced by executing the reference graph templates (tests/golden/make_golden.py).

This pins the oracle before it is trusted as the checker of the HIP engine.
"""
import os

import numpy as np
import pytest
import torch

from genie_tts_amd import synth, weights as W

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.fixture(scope="module", autouse=True)
def exact_div_term():
    from oracle import restate as R
    R.set_div_term(np.load(os.path.join(GOLD, "pe_div_term.npy")))
    yield
    R.set_div_term(None)


def fingerprint(w):
    return np.array([float(np.abs(np.asarray(w[k], np.float64)).sum()) for k in sorted(w)])


def test_synthetic_weight_generator_is_pinned():
    fp = gold("weights_fingerprint.npz")
    np.testing.assert_array_equal(fingerprint(synth.synth_weights(W.t2s_encoder_spec(), fp16=False)), fp["t2s_encoder"])
    np.testing.assert_array_equal(fingerprint(synth.synth_weights(W.t2s_spec())), fp["t2s"])
    np.testing.assert_array_equal(fingerprint(synth.synth_weights(W.vits_spec("v2"))), fp["vits_v2"])
    np.testing.assert_array_equal(fingerprint(synth.synth_weights(W.vits_spec("v2ProPlus"))), fp["vits_v2pp"])
    np.testing.assert_array_equal(fingerprint(synth.synth_weights(W.prompt_encoder_spec())), fp["prompt_encoder"])


@pytest.fixture(scope="module")
def t2s_model():
    from oracle import restate as R
    w = synth.synthetic_character("v2")
    return w, R.T2SModel(w["t2s"])


@pytest.mark.parametrize("case", ["t2s_small.npz", "t2s_nominal.npz"])
def test_t2s_restatement_vs_graphs(t2s_model, case):
    from oracle import restate as R
    g = gold(case)
    w, m = t2s_model
    R_, S_ = g["ref_seq"].shape[1], g["text_seq"].shape[1]
    x, prompts = R.t2s_encoder(w["t2s_encoder"], g["ref_seq"], g["text_seq"], np.zeros((R_, 1024), np.float32),
                               np.zeros((S_, 1024), np.float32), g["ssl"])
    np.testing.assert_array_equal(prompts.numpy(), g["prompts"])
    np.testing.assert_allclose(x.numpy(), g["x"], atol=2e-5)
    st, lg = R.t2s_prefill(m, x, prompts.numpy(), torch.ones(1025))
    assert st.y == g["y_prefill"].reshape(-1).tolist()
    np.testing.assert_allclose(lg.numpy(), g["prefill_logits"].reshape(-1), atol=2e-4)
    np.testing.assert_allclose(st.k[0].numpy(), g["kv_k0"], atol=1e-4)
    for i in range(len(g["step_tokens"])):
        stop, lg = R.t2s_step(m, st, torch.ones(1025))
        np.testing.assert_allclose(lg.numpy(), g["step_logits"][i].reshape(-1), atol=5e-4)
        assert st.y[-1] == int(g["step_tokens"][i])
        assert bool(stop) == bool(g["stops"][i])
    sem = R.trim_tokens(st.y, int(g["loop_idx"]))
    np.testing.assert_array_equal(sem, g["pred_semantic"])


def test_t2s_forced_eos_returns_prompts(t2s_model):
    """Stop at loop index 0: y[:, -0:] is the whole y; after the >=1024 filter the
    output equals the prompts (Inference.py:41-44,108-109)."""
    from oracle import restate as R
    g = gold("t2s_eos.npz")
    w, _ = t2s_model
    w_eos = dict(w["t2s"])
    b = np.asarray(w_eos["transformer_encoder.layers.23.norm2.bias"], np.float32)
    w_eos["transformer_encoder.layers.23.norm2.weight"] = np.full(512, 1e-3, np.float16)
    pred = np.asarray(w_eos["ar_predict_layer.weight"], np.float32).copy()
    pred[1024] = 10.0 * b
    w_eos["ar_predict_layer.weight"] = pred.astype(np.float16)
    m = R.T2SModel(w_eos)
    sem, st, prompts = R.t2s_generate(w["t2s_encoder"], m, g["ref_seq"], np.zeros((12, 1024), np.float32),
                                      g["text_seq"], np.zeros((10, 1024), np.float32), g["ssl"])
    np.testing.assert_array_equal(sem, g["pred_semantic"])
    np.testing.assert_array_equal(sem.reshape(-1), prompts.numpy().reshape(-1))


@pytest.mark.parametrize("ver", ["v2", "v2ProPlus"])
def test_vits_restatement_vs_graphs(ver):
    from oracle import restate as R
    g = gold(f"vits_{ver}.npz")
    vm = R.VitsModel(synth.synth_weights(W.vits_spec(ver)), ver)
    kw = dict(ref_audio=g["ref_audio"]) if ver == "v2" else dict(ge=g["ge"], ge_advanced=g["ge_advanced"])
    a0 = vm(g["text_seq"], g["pred_semantic"], **kw).numpy()
    np.testing.assert_allclose(vm.last["m_p"].numpy(), g["m_p"], atol=2e-5)
    np.testing.assert_allclose(vm.last["logs_p"].numpy(), g["logs_p"], atol=2e-5)
    if ver == "v2":
        np.testing.assert_allclose(vm.last["ge"].numpy(), g["ge"], atol=2e-5)
    assert np.sqrt(np.mean((a0 - g["audio_zero"]) ** 2)) < 1e-5
    a1 = vm(g["text_seq"], g["pred_semantic"], eps=g["eps"], **kw).numpy()
    assert np.sqrt(np.mean((a1 - g["audio_eps"]) ** 2)) < 1e-5
    assert a0.shape == (1280 * g["pred_semantic"].shape[-1],)


def test_prompt_encoder_restatement_vs_graph():
    from oracle import restate as R
    g = gold("prompt_encoder.npz")
    ge, ga = R.prompt_encoder(synth.synth_weights(W.prompt_encoder_spec()), g["ref_audio"], g["sv_emb"])
    np.testing.assert_allclose(ge.numpy(), g["ge"], atol=2e-5)
    np.testing.assert_allclose(ga.numpy(), g["ge_advanced"], atol=2e-5)


@pytest.mark.parametrize("case", ["t2s_nominal81.npz", "t2s_sampled81.npz"])
def test_t2s_restatement_bench_size_vs_graphs(t2s_model, case):
    """The bench's 81-step nominal utterance, greedy and top-k 15 sampled with the
    engine's Philox q (tests/golden/make_golden_bench.py), both pinned to the graphs."""
    from oracle import restate as R
    from tests.philox import sampler_noise
    g, nom = gold(case), gold("t2s_nominal.npz")
    w, m = t2s_model
    seed = int(g["seed"])
    q_fn = None if seed == 0 else (lambda idx: torch.from_numpy(sampler_noise(1025, idx + 1, 0, seed)))
    R_, S_ = nom["ref_seq"].shape[1], nom["text_seq"].shape[1]
    sem, st, _ = R.t2s_generate(w["t2s_encoder"], m, nom["ref_seq"], np.zeros((R_, 1024), np.float32),
                                nom["text_seq"], np.zeros((S_, 1024), np.float32), nom["ssl"],
                                R.SamplerCfg(top_k=int(g["top_k"])), force_steps=len(g["step_tokens"]), q_fn=q_fn)
    P1 = g["y_prefill"].shape[1]
    assert st.y[:P1] == g["y_prefill"].reshape(-1).tolist()
    assert st.y[P1:] == g["step_tokens"].tolist()
    np.testing.assert_array_equal(sem, g["pred_semantic"])


@pytest.mark.parametrize("ver", ["v2", "v2ProPlus"])
def test_vits_restatement_bench_size_vs_graphs(ver):
    """G=80 (the bench's 102,400 samples), zero noise and the engine's Philox eps."""
    from oracle import restate as R
    from tests.philox import vits_noise
    g = gold(f"vits_{ver}_g80.npz")
    vm = R.VitsModel(synth.synth_weights(W.vits_spec(ver)), ver)
    kw = dict(ref_audio=g["ref_audio"]) if ver == "v2" else dict(ge=g["ge"], ge_advanced=g["ge_advanced"])
    G = g["pred_semantic"].shape[-1]
    a0 = vm(g["text_seq"], g["pred_semantic"], **kw).numpy()
    assert np.sqrt(np.mean((a0 - g["audio_zero"]) ** 2)) < 1e-5
    eps = vits_noise(192 * 2 * G, int(g["noise_seed"])).reshape(1, 192, 2 * G)
    a1 = vm(g["text_seq"], g["pred_semantic"], eps=eps, **kw).numpy()
    assert np.sqrt(np.mean((a1 - g["audio_philox"]) ** 2)) < 1e-5
