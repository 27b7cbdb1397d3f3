"""GPU: the V2ProPlus speaker-verification model on the engine (gsv_sv, sv.hip) against
the oracle's restatement of GPT-SoVITS's SV (Kaldi fbank -> ERes2NetV2.forward3,
oracle/sv.py) on the same synthetic fp32 weights.  ONNX-level parity is unpinned
(speaker_encoder.onnx is absent); the bar is the fp32 model within the split-fp16
MFMA's accuracy (and the f32 MFMA path's): RMS <= 1e-4 x max(1, std) of the 20480-d
embedding."""
import numpy as np
import pytest

from genie_tts_amd import synth

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4


@pytest.fixture(scope="module")
def svm():
    from genie_tts_amd.engine import Engine
    w = synth.synth_sv_weights()
    e = Engine({"sv": w}, "v2")
    yield e, w
    e.close()


def _clip(n, tag):
    """Speech-like test signal: two tones under noise, then the reference's 0.3 s of silence."""
    r = synth.rng_for(tag)
    t = np.arange(n) / 16000.0
    a = 0.3 * np.sin(2 * np.pi * 220 * t) + 0.1 * np.sin(2 * np.pi * 1330 * t) + 0.05 * r.standard_normal(n)
    a[max(0, n - 4800):] = 0.0
    return a.astype(np.float32)


def _check(got, ref):
    assert got.shape == ref.shape == (1, 20480)
    rms = float(np.sqrt(np.mean((got - ref) ** 2)))
    print(f"rms {rms:.2e} max {np.abs(got - ref).max():.2e} ref std {ref.std():.3f}")
    assert rms <= RMS_TOL * max(1.0, float(ref.std())), rms


# 400 samples = one fbank frame (the minimum); a ragged 1 s; the nominal 5.3 s reference
# clip + 0.3 s of silence at 16 kHz; a 30 s clip (2998 frames)
@pytest.mark.parametrize("n", [400, 16077, 89600, 480000])
def test_sv_vs_oracle(svm, n):
    from oracle import sv as S
    e, w = svm
    a = _clip(n, f"sv-{n}") if n > 4800 else (0.2 * synth.rng_for("sv-min").standard_normal(n)).astype(np.float32)
    _check(e.sv(a).cpu().numpy(), S.sv_embedding(w, a))


def test_sv_f32_path_vs_oracle(svm):
    """Option sv_f16 = 0: every conv on the f32 MFMA (no fp16 split) -- same bar."""
    from oracle import sv as S
    e, w = svm
    a = _clip(16077, "sv-f32")
    e.set_option("sv_f16", 0)
    try:
        got = e.sv(a).cpu().numpy()
    finally:
        e.set_option("sv_f16", 1)
    _check(got, S.sv_embedding(w, a))


def test_sv_fp16_range_fallback(svm):
    """An activation beyond the fp16 range (limit lowered to 1 here) sets the flag and the
    call runs again on the f32 path: the result is that path's, bit for bit."""
    e, _ = svm
    a = _clip(16077, "sv-ovf")
    e.set_option("sv_f16", 0)
    try:
        want = e.sv(a).cpu().numpy()
    finally:
        e.set_option("sv_f16", 1)
    before = e.counter("sv_f32_reruns")
    e.set_option("sv_f16_limit", 1)
    try:
        got = e.sv(a).cpu().numpy()
    finally:
        e.set_option("sv_f16_limit", 0)
    assert e.counter("sv_f32_reruns") == before + 1
    assert np.array_equal(got, want)


def test_sv_too_short(svm):
    from genie_tts_amd.engine import EngineError
    e, _ = svm
    with pytest.raises(EngineError):
        e.sv(np.zeros(399, np.float32))


def test_sv_repeatable(svm):
    e, _ = svm
    a = _clip(32000, "sv-rep")
    assert np.array_equal(e.sv(a).cpu().numpy(), e.sv(a).cpu().numpy())


def test_reference_audio_gets_sv_from_engine(svm, tmp_path):
    """V2ProPlus: set_reference_audio(path) without sv_emb, then tts() runs the engine's SV
    on the clip's 16 kHz copy (ReferenceAudio.update_global_emb, ReferenceAudio.py:68-76);
    the embedding matches the oracle and the audio equals a call given that sv_emb."""
    import wave
    import genie_tts_amd as genie
    from genie_tts_amd.api import _reference_audios
    from genie_tts_amd.engine import make_sampler
    from genie_tts_amd.model_manager import build_model, model_manager
    from genie_tts_amd.sessions import SvSession
    from oracle import sv as S
    e, w = svm
    cw = dict(synth.synthetic_character("v2ProPlus"))
    t2s = dict(cw["t2s"])          # forced EOS (tests/golden/make_golden.py): a short utterance
    b = np.asarray(t2s["transformer_encoder.layers.23.norm2.bias"], np.float32)
    t2s["transformer_encoder.layers.23.norm2.weight"] = np.full(512, 1e-3, np.float16)
    pred = np.asarray(t2s["ar_predict_layer.weight"], np.float32).copy()
    pred[1024] = 10.0 * b
    t2s["ar_predict_layer.weight"] = pred.astype(np.float16)
    cw["t2s"] = t2s
    m = build_model(cw, "v2ProPlus", sampler=make_sampler(greedy=True))
    m.VITS.noise = "zero"
    model_manager._put("svc", m)
    model_manager.character_to_language["svc"] = "Japanese"
    wav_path = str(tmp_path / "ref.wav")
    x = np.concatenate([_clip(2 * 16000, "sv-wav")] * 2).clip(-1, 1)     # 2 s at 32 kHz
    with wave.open(wav_path, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(32000)
        wf.writeframes((x * 32767).astype("<i2").tobytes())
    model_manager.speaker_verification_model = SvSession(e)
    txt = synth.synth_phones(10, "sv-t")
    try:
        genie.set_reference_audio("svc", wav_path, "", "Japanese", phonemes_seq=synth.synth_phones(12, "sv-r"),
                                  ssl_content=synth.synth_ssl(61, "sv-s"))
        out = genie.tts("svc", txt, split_sentence=False)
        ref = _reference_audios["svc"]
        assert ref.sv_emb is not None and ref.sv_emb.shape == (1, 20480)
        _check(ref.sv_emb, S.sv_embedding(w, ref.audio_16k))
        sv = ref.sv_emb.copy()
        genie.clear_reference_audio_cache()
        genie.set_reference_audio("svc", wav_path, "", "Japanese", phonemes_seq=synth.synth_phones(12, "sv-r"),
                                  ssl_content=synth.synth_ssl(61, "sv-s"), sv_emb=sv)
        again = genie.tts("svc", txt, split_sentence=False)
        assert out.size > 0 and np.array_equal(out, again)
    finally:
        model_manager.speaker_verification_model = None
        model_manager.character_to_model.pop("svc", None)
        genie.clear_reference_audio_cache()


@pytest.mark.parametrize("folded", [False, True])
def test_sv_renamed_export_on_the_engine(svm, tmp_path, folded):
    """An export with renamed initializers (weights.load_sv_weights' Conv-order mapping):
    with BatchNormalization nodes the engine gets the very same tensors; with BatchNorm
    folded into the convs it takes their biases instead and gives the same embedding
    (the engine folds BatchNorm in the same fp32 arithmetic)."""
    from genie_tts_amd import weights as W
    from genie_tts_amd.engine import Engine
    from tests.sv_export import export
    e0, w = svm
    p = str(tmp_path / "speaker_encoder.onnx")
    export(w, p, folded=folded)
    e = Engine({"sv": W.load_sv_weights(p)}, "v2")
    try:
        a = _clip(48000, "sv-renamed")
        got, ref = e.sv(a).cpu().numpy().reshape(1, -1), e0.sv(a).cpu().numpy().reshape(1, -1)
        rel = float(np.sqrt(np.mean((got - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))
        print(f"folded={folded}: rel rms {rel:.2e}")
        assert rel <= 1e-6, rel
    finally:
        e.close()
