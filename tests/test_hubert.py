"""CPU: the CN-HuBERT weight layout and frame arithmetic against transformers'
HubertModel (the published model behind chinese-hubert-base.onnx,
ReferenceAudio.py:48-52; the oracle is oracle/hubert.py)."""
import numpy as np

from genie_tts_amd import weights as W


def _hf():
    from oracle import hubert as H
    from genie_tts_amd import synth
    return H, H.hubert_model(synth.synth_weights(W.hubert_spec()))


def test_spec_matches_hubert_model_state_dict():
    H, m = _hf()
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    spec = W.hubert_spec()
    for k, shape in spec.items():
        if k == "encoder.pos_conv_embed.conv.weight":
            v = [s for n, s in sd.items() if "pos_conv_embed.conv" in n and ("original1" in n or n.endswith("weight_v"))]
            assert v and v[0] == shape
            continue
        assert sd[k] == shape, k
    extra = {k for k in sd if k not in spec and "pos_conv_embed.conv" not in k}
    assert extra == {"masked_spec_embed"}   # used only with time masking (training)


def test_frame_count_matches_model():
    from genie_tts_amd import engine
    H, m = _hf()
    import torch
    for n in (400, 16000, 24000, 84800, 84801):
        want = int(m._get_feat_extract_output_lengths(torch.tensor(n)))
        lib = engine.lib()
        assert lib.gsv_hubert_frames(n) == want, n


def test_oracle_reproduces_folded_pos_conv_weight():
    """v = W, g = ||W|| per tap gives back W through the weight-norm parametrization."""
    import torch
    H, m = _hf()
    from genie_tts_amd import synth
    w = synth.synth_weights(W.hubert_spec())
    got = m.encoder.pos_conv_embed.conv.weight.detach().numpy()
    np.testing.assert_allclose(got, np.asarray(w["encoder.pos_conv_embed.conv.weight"], np.float32), rtol=1e-5,
                               atol=1e-7)
    x = (0.1 * synth.rng_for("hb-cpu").standard_normal(8000)).astype(np.float32)
    out = H.ssl_content(m, x)
    assert out.shape == (1, 768, 24) and np.isfinite(out).all()


def test_input_normalisation_variants_differ():
    """The raw-clip input (GPT-SoVITS inference, Genie ReferenceAudio.py:48-52; the engine's
    gsv_hubert) and CNHubert.forward's normalised input give different features: the
    oracle keeps both, the engine implements the raw one (tests/test_hubert_gpu.py);
    the two differ beyond the parity bar, so the choice is not cosmetic."""
    H, m = _hf()
    from genie_tts_amd import synth
    x = (0.05 * synth.rng_for("hb-norm").standard_normal(8000) + 0.01).astype(np.float32)
    raw, nrm = H.ssl_content(m, x), H.ssl_content(m, x, normalize=True)
    n = H.feature_normalize(x)
    assert abs(float(n.mean())) < 1e-5 and abs(float(n.std()) - 1.0) < 1e-3
    assert raw.shape == nrm.shape
    # the first conv layer's GroupNorm absorbs most of the rescaling, but not all:
    # ~2e-3 RMS here, 20x the 1e-4 parity bar
    assert float(np.sqrt(np.mean((raw - nrm) ** 2))) > 1e-3
