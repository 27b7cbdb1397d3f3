"""GPU: CN-HuBERT on the engine (gsv_hubert, hubert.hip) against the oracle,
transformers' HubertModel on the same synthetic weights (oracle/hubert.py).
ONNX-level parity is unpinned (chinese-hubert-base.onnx is absent); the bar is
the published model's fp32 output within split-fp16 GEMM accuracy."""
import numpy as np
import pytest

from genie_tts_amd import synth, weights as W

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4


@pytest.fixture(scope="module")
def hub():
    from genie_tts_amd.engine import Engine
    from oracle import hubert as H
    w = synth.synth_weights(W.hubert_spec())
    e = Engine({"hubert": w}, "v2")
    yield e, H, H.hubert_model(w), w
    e.close()


@pytest.mark.parametrize("n", [24000, 84800])   # 1.5 s; the nominal 5.3 s reference
def test_hubert_vs_transformers(hub, n):
    e, H, m, _ = hub
    a = (0.1 * synth.rng_for(f"hb-{n}").standard_normal(n)).astype(np.float32)
    got = e.hubert(a).cpu().numpy()
    ref = H.ssl_content(m, a)[0]
    assert got.shape == ref.shape
    rms = float(np.sqrt(np.mean((got - ref) ** 2)))
    print(f"n={n} T={got.shape[1]} rms {rms:.2e} max {np.abs(got - ref).max():.2e} ref std {ref.std():.3f}")
    assert rms <= RMS_TOL * max(1.0, float(ref.std())), rms


def test_hubert_session_and_reference_audio(hub, tmp_path):
    """set_reference_audio without ssl_content runs the engine's CN-HuBERT on the
    clip's 16 kHz copy (ReferenceAudio.py:43-52)."""
    import wave
    import genie_tts_amd as genie
    from genie_tts_amd.model_manager import model_manager
    from genie_tts_amd.sessions import HubertSession
    e, H, m, w = hub
    sess = HubertSession(e)
    a = (0.1 * synth.rng_for("hb-sess").standard_normal((1, 16000))).astype(np.float32)
    (ssl,) = sess.run(None, {"input_values": a})
    assert ssl.shape == (1, 768, 49)
    from tests.test_tutorial_gpu import toy_g2p
    from tests.test_api_gpu import _eos_character
    genie.load_weights("hb", _eos_character(), "v2")
    wav_path = str(tmp_path / "ref.wav")
    x = (0.2 * synth.rng_for("hb-wav").standard_normal(3 * 32000)).clip(-1, 1)
    with wave.open(wav_path, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(32000)
        wf.writeframes((x * 32767).astype("<i2").tobytes())
    genie.set_g2p(toy_g2p)
    model_manager.cn_hubert = sess
    try:
        genie.set_reference_audio("hb", wav_path, "こんにちは。", "Japanese")
        from genie_tts_amd.api import _reference_audios
        ref = _reference_audios["hb"]
        want = H.ssl_content(m, ref.audio_16k)
        assert ref.ssl_content.shape == want.shape
        rms = float(np.sqrt(np.mean((ref.ssl_content - want) ** 2)))
        assert rms <= RMS_TOL * max(1.0, float(want.std())), rms
    finally:
        model_manager.cn_hubert = None
        genie.set_g2p(None)
        genie.unload_character("hb")
        genie.clear_reference_audio_cache()


def test_hubert_fp32_weights_vs_transformers():
    """load_cn_hubert(model_path) without the fp16 bin loads a plain fp32 graph
    (ModelManager.py:183-187): fp32-valued weights run on the split-weight GEMMs."""
    from genie_tts_amd.engine import Engine
    from oracle import hubert as H
    w = synth.synth_weights(W.hubert_spec(), fp16=False)
    e = Engine({"hubert": w}, "v2")
    try:
        assert e.counter("w16_split_tensors") == 6 + 2 + 4 * 12   # convs 1-6, projection, pos conv, layers
        a = (0.1 * synth.rng_for("hb-f32").standard_normal(24000)).astype(np.float32)
        got = e.hubert(a).cpu().numpy()
        ref = H.ssl_content(H.hubert_model(w), a)[0]
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"fp32 weights: rms {rms:.2e} ref std {ref.std():.3f}")
        assert rms <= RMS_TOL * max(1.0, float(ref.std())), rms
    finally:
        e.close()
