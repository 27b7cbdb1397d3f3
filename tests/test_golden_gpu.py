"""GPU: the HIP engine (via the C ABI) against the golden fixtures produced by
executing the reference graph templates (tests/golden/make_golden.py).

Bars: greedy token ids bit-exact; logits/KV within fp32 reduction-order noise;
waveform RMS <= 1e-4 (north_star)."""
import os

import numpy as np
import pytest

from genie_tts_amd import synth, weights as W

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.fixture(scope="module")
def div():
    return np.load(os.path.join(GOLD, "pe_div_term.npy"))


def _eng(groups, ver, div):
    from genie_tts_amd.engine import Engine
    return Engine(groups, ver, pe_div_term=div)


@pytest.mark.parametrize("case", ["t2s_small.npz", "t2s_nominal.npz"])
def test_t2s_vs_reference_graphs(case, div):
    from genie_tts_amd.engine import make_sampler
    g = gold(case)
    w = synth.synthetic_character("v2")
    e = _eng({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2", div)
    x, prompts = e.t2s_encode(g["ref_seq"], g["text_seq"], None, None, g["ssl"])
    np.testing.assert_array_equal(prompts.cpu().numpy(), g["prompts"].reshape(-1))
    np.testing.assert_allclose(x.cpu().numpy(), g["x"].reshape(-1, 512), atol=2e-5)
    y, lg = e.t2s_prefill(g["x"].reshape(-1, 512), g["prompts"])
    np.testing.assert_array_equal(y.cpu().numpy(), g["y_prefill"].reshape(-1))
    np.testing.assert_allclose(lg.cpu().numpy(), g["prefill_logits"].reshape(-1), atol=2e-4)
    k0, v0 = e.t2s_read_kv(0)
    np.testing.assert_allclose(k0.cpu().numpy(), g["kv_k0"], atol=1e-4)
    n = len(g["step_tokens"])
    y2, stop, lgs = e.t2s_decode_steps(n)
    P1 = g["y_prefill"].shape[1]
    np.testing.assert_array_equal(y2[P1:P1 + n].cpu().numpy(), g["step_tokens"])
    np.testing.assert_array_equal(stop.cpu().numpy().astype(bool), g["stops"])
    np.testing.assert_allclose(lgs.cpu().numpy(), g["step_logits"].reshape(n, -1), atol=5e-4)
    out = e.t2s_generate([(g["ref_seq"], g["text_seq"], None, None, g["ssl"])], make_sampler(force_steps=n))
    np.testing.assert_array_equal(out[0], g["pred_semantic"].reshape(-1))
    e.close()


def test_t2s_forced_eos_vs_reference_graphs(div):
    from genie_tts_amd.engine import make_sampler
    g = gold("t2s_eos.npz")
    w = synth.synthetic_character("v2")
    t2s = dict(w["t2s"])
    b = np.asarray(t2s["transformer_encoder.layers.23.norm2.bias"], np.float32)
    t2s["transformer_encoder.layers.23.norm2.weight"] = np.full(512, 1e-3, np.float16)
    pred = np.asarray(t2s["ar_predict_layer.weight"], np.float32).copy()
    pred[1024] = 10.0 * b
    t2s["ar_predict_layer.weight"] = pred.astype(np.float16)
    e = _eng({"t2s_encoder": w["t2s_encoder"], "t2s": t2s}, "v2", div)
    out = e.t2s_generate([(g["ref_seq"], g["text_seq"], None, None, g["ssl"])], make_sampler())
    np.testing.assert_array_equal(out[0], g["pred_semantic"].reshape(-1))
    np.testing.assert_array_equal(out[0], g["prompts"].reshape(-1))
    e.close()


@pytest.mark.parametrize("ver", ["v2", "v2ProPlus"])
def test_vits_vs_reference_graphs(ver, div):
    g = gold(f"vits_{ver}.npz")
    w = synth.synthetic_character(ver)
    e = _eng({k: w[k] for k in w}, ver, div)
    kw = dict(ref_audio=g["ref_audio"]) if ver == "v2" else dict(ge=g["ge"], ge_advanced=g["ge_advanced"])
    a0 = e.vits_decode(g["text_seq"], g["pred_semantic"], **kw).cpu().numpy()
    a1 = e.vits_decode(g["text_seq"], g["pred_semantic"], eps=g["eps"], **kw).cpu().numpy()
    for got, ref in ((a0, g["audio_zero"]), (a1, g["audio_eps"])):
        assert got.shape == ref.shape
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        assert rms <= 1e-4, rms
    if ver == "v2ProPlus":
        p = gold("prompt_encoder.npz")
        ge, ga = e.prompt_encode(p["ref_audio"], p["sv_emb"])
        np.testing.assert_allclose(ge.cpu().numpy(), p["ge"].reshape(-1), atol=2e-4)
        np.testing.assert_allclose(ga.cpu().numpy(), p["ge_advanced"].reshape(-1), atol=2e-4)
    e.close()


@pytest.mark.parametrize("case", ["t2s_nominal81.npz", "t2s_sampled81.npz"])
def test_t2s_bench_size_vs_reference_graphs(case, div):
    """The bench workload itself (configs[1]: 81 loop steps), greedy and top-k 15
    sampled with the Philox q the graphs were run with (make_golden_bench.py):
    every token bit-exact, through the persistent decode of gsv_t2s_generate."""
    from genie_tts_amd.engine import make_sampler
    g, nom = gold(case), gold("t2s_nominal.npz")
    w = synth.synthetic_character("v2")
    e = _eng({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2", div)
    seed = int(g["seed"])
    n = len(g["step_tokens"])
    smp = make_sampler(top_k=int(g["top_k"]), greedy=seed == 0, seed=seed or 1234, force_steps=n)
    out = e.t2s_generate([(nom["ref_seq"], nom["text_seq"], None, None, nom["ssl"])], smp)
    np.testing.assert_array_equal(out[0], g["pred_semantic"].reshape(-1))
    # Inference.py:108: y[:, -idx:] with idx = n - 1 and the last token zeroed
    np.testing.assert_array_equal(out[0][:n - 2], g["step_tokens"][1:n - 1])
    e.close()


@pytest.mark.parametrize("ver", ["v2", "v2ProPlus"])
def test_vits_bench_size_vs_reference_graphs(ver, div):
    """G=80 (102,400 samples, the bench's utterance): zero noise and the device
    Philox eps (noise_seed) against the graphs run with the same eps."""
    g = gold(f"vits_{ver}_g80.npz")
    w = synth.synthetic_character(ver)
    e = _eng({k: w[k] for k in w}, ver, div)
    kw = dict(ref_audio=g["ref_audio"]) if ver == "v2" else dict(ge=g["ge"], ge_advanced=g["ge_advanced"])
    a0 = e.vits_decode(g["text_seq"], g["pred_semantic"], **kw).cpu().numpy()
    a1 = e.vits_decode(g["text_seq"], g["pred_semantic"], noise_seed=int(g["noise_seed"]), **kw).cpu().numpy()
    for got, ref in ((a0, g["audio_zero"]), (a1, g["audio_philox"])):
        assert got.shape == ref.shape == (102400,)
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        assert rms <= 1e-4, rms
    e.close()
