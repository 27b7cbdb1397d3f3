"""GPU: the drop-in surface (session objects, GENIE driver, genie_tts-style API)
on top of the C ABI, against the oracle and the golden fixtures.

- The reference's own session-by-session loop (GENIE.t2s_cpu, Inference.py:63-109)
  run over the engine-backed sessions and the one-call device path (GENIE.t2s)
  give identical token ids, equal to the fixture made from the reference graphs.
- api.tts end to end equals oracle/restate.py (waveform RMS <= 1e-4).
"""
import os

import numpy as np
import pytest

from genie_tts_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _eos_character():
    """Forced-EOS weights of tests/golden/make_golden.py (stop fires at idx 0)."""
    w = dict(synth.synthetic_character("v2"))
    t2s = dict(w["t2s"])
    b = np.asarray(t2s["transformer_encoder.layers.23.norm2.bias"], np.float32)
    t2s["transformer_encoder.layers.23.norm2.weight"] = np.full(512, 1e-3, np.float16)
    pred = np.asarray(t2s["ar_predict_layer.weight"], np.float32).copy()
    pred[1024] = 10.0 * b
    t2s["ar_predict_layer.weight"] = pred.astype(np.float16)
    w["t2s"] = t2s
    return w


@pytest.fixture(scope="module")
def model():
    from genie_tts_amd.engine import make_sampler
    from genie_tts_amd.model_manager import build_model
    div = np.load(os.path.join(GOLD, "pe_div_term.npy"))
    w = _eos_character()
    m = build_model(w, "v2", sampler=make_sampler(greedy=True), pe_div_term=div)
    m.VITS.noise = "zero"          # deterministic vocoder: parity against the oracle with eps = 0
    yield m, w
    m.ENGINE.close()


def test_session_names_follow_templates(model):
    m, _ = model
    names = [i.name for i in m.T2S_STAGE_DECODER.get_inputs()]
    assert names[:4] == ["iy", "iy_emb", "past_k_layer_0", "past_v_layer_0"] and names[-1] == "past_v_layer_23"
    outs = [o.name for o in m.T2S_STAGE_DECODER.get_outputs()]
    assert outs[:3] == ["y", "y_emb", "stop_condition_tensor"] and len(outs) == 51


def test_reference_loop_and_device_path_agree_with_golden(model):
    from genie_tts_amd.inference import GENIE, eos_filter
    m, _ = model
    g = dict(np.load(os.path.join(GOLD, "t2s_eos.npz"), allow_pickle=False))
    zr = np.zeros((g["ref_seq"].shape[1], 1024), np.float32)
    zt = np.zeros((g["text_seq"].shape[1], 1024), np.float32)
    gen = GENIE()
    sem_loop = gen.t2s_cpu(g["ref_seq"], zr, g["text_seq"], zt, g["ssl"], m.T2S_ENCODER,
                           m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER)
    sem_loop = eos_filter(sem_loop)
    sem_dev = gen.t2s(g["ref_seq"], zr, g["text_seq"], zt, g["ssl"], m.ENGINE, m.T2S_FIRST_STAGE_DECODER.sampler)
    np.testing.assert_array_equal(sem_loop, g["pred_semantic"])
    np.testing.assert_array_equal(sem_dev, g["pred_semantic"])


def test_session_outputs_match_golden_shapes(model):
    m, _ = model
    g = dict(np.load(os.path.join(GOLD, "t2s_eos.npz"), allow_pickle=False))
    x, prompts = m.T2S_ENCODER.run(None, {"ref_seq": g["ref_seq"], "text_seq": g["text_seq"],
                                          "ref_bert": np.zeros((12, 1024), np.float32),
                                          "text_bert": np.zeros((10, 1024), np.float32),
                                          "ssl_content": g["ssl"]})
    assert x.shape == g["x"].shape and prompts.shape == g["prompts"].shape
    np.testing.assert_array_equal(prompts, g["prompts"])
    y, y_emb, *kv = m.T2S_FIRST_STAGE_DECODER.run(None, {"x": x, "prompts": prompts})
    L, P = x.shape[1], prompts.shape[1]
    assert y.shape == (1, P + 1) and y_emb.shape == (1, P, 512) and len(kv) == 48
    assert kv[0].shape == (L + P, 1, 512)
    names = [i.name for i in m.T2S_STAGE_DECODER.get_inputs()]
    y2, e2, stop, *kv2 = m.T2S_STAGE_DECODER.run(None, dict(zip(names, [y, y_emb, *kv])))
    assert y2.shape == (1, P + 2) and e2.shape == (1, P + 1, 512) and kv2[0].shape == (L + P + 1, 1, 512)
    assert stop.dtype == np.bool_ and stop.shape == ()
    from genie_tts_amd.sessions import SessionStateError
    with pytest.raises(SessionStateError):
        m.T2S_STAGE_DECODER.run(None, dict(zip(names, [y, y_emb, *kv])))   # stale input


def test_api_tts_end_to_end(model):
    import genie_tts_amd as G
    from genie_tts_amd import api
    from genie_tts_amd.model_manager import model_manager
    from oracle import restate as R
    m, w = model
    model_manager._put("eos_char", m)
    model_manager.character_to_language["eos_char"] = "Japanese"
    ref = synth.synth_phones(12, "api-r")
    txt = synth.synth_phones(10, "api-t")
    ssl = synth.synth_ssl(41, "api-s")
    audio32 = synth.synth_ref_audio(32000 * 2, "api-a")
    G.set_reference_features("eos_char", ref, None, audio32, ssl)
    out = G.tts("eos_char", txt, split_sentence=False, sampler=m.T2S_FIRST_STAGE_DECODER.sampler)
    div = np.load(os.path.join(GOLD, "pe_div_term.npy"))
    R.set_div_term(div)
    try:
        tm = R.T2SModel(w["t2s"])
        z = lambda n: np.zeros((n, 1024), np.float32)
        sem, _, _ = R.t2s_generate(w["t2s_encoder"], tm, ref, z(12), txt, z(10), ssl)
        ref_audio = R.VitsModel(w["vits"], "v2")(txt, np.asarray(sem).reshape(1, 1, -1), ref_audio=audio32)
    finally:
        R.set_div_term(None)
    ref_audio = ref_audio.numpy().reshape(-1)
    assert out.shape == ref_audio.shape
    assert float(np.sqrt(np.mean((out - ref_audio) ** 2))) <= 1e-4
    model_manager.character_to_model.pop("eos_char", None)
    api.clear_reference_audio_cache()


@pytest.mark.parametrize("lens", [(10, 17, 25), (10, 17, 25, 8, 13, 21)])
def test_tts_batch_equals_single(model, lens):
    """3 or 6 sentences: one batched generate on the multi-sequence persistent decode
    (GENIE.tts_batch_t2s); every sentence's audio equals its own single-sentence call."""
    from genie_tts_amd.inference import GENIE, ReferenceAudio
    m, _ = model
    ref = ReferenceAudio(phonemes_seq=synth.synth_phones(12, "b-r"), text_bert=np.zeros((12, 1024), np.float32),
                         audio_32k=synth.synth_ref_audio(32000 * 2, "b-a").reshape(1, -1),
                         ssl_content=synth.synth_ssl(41, "b-s").reshape(1, 768, -1))
    texts = [synth.synth_phones(n, f"b-t{n}") for n in lens]
    gen = GENIE()
    sp = m.T2S_FIRST_STAGE_DECODER.sampler
    batch = gen.tts_batch([(t, None) for t in texts], ref, m, sp)
    for t, b in zip(texts, batch):
        single = gen.tts(t, ref, m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER, m.VITS, None,
                         sampler=sp)
        assert single.shape == b.shape
        # the batch's vocoder runs one generator pass over all sentences (seg_vocoder):
        # equal to the single calls to fp32 rounding
        rel = float(np.sqrt(np.mean((single - b) ** 2)) / np.sqrt(np.mean(single ** 2)))
        assert rel <= 1e-5 and np.abs(single - b).max() <= 1e-4, rel


def test_tts_stream_equals_single(model):
    """GENIE.tts_stream (vocoder of sentence i overlapped with the T2S of sentence
    i+1 on split CUs) yields what tts gives sentence by sentence."""
    from genie_tts_amd.inference import GENIE, ReferenceAudio
    m, _ = model
    ref = ReferenceAudio(phonemes_seq=synth.synth_phones(12, "s-r"), text_bert=np.zeros((12, 1024), np.float32),
                         audio_32k=synth.synth_ref_audio(32000 * 2, "s-a").reshape(1, -1),
                         ssl_content=synth.synth_ssl(41, "s-s").reshape(1, 768, -1))
    texts = [synth.synth_phones(n, f"s-t{n}") for n in (10, 17, 25, 12)]
    gen = GENIE()
    sp = m.T2S_FIRST_STAGE_DECODER.sampler
    args = (ref, m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER, m.VITS, None)
    try:
        streamed = list(gen.tts_stream(texts, *args, sampler=sp, vocoder_cus=64))
    finally:
        m.ENGINE.set_vocoder_cus(0)
    assert len(streamed) == len(texts)
    for t, a in zip(texts, streamed):
        single = gen.tts(t, *args, sampler=sp)
        assert single.shape == a.shape
        np.testing.assert_allclose(single, a, atol=1e-6)


def test_tts_stream_abandoned_leaves_the_engine_clean(model):
    """A stream closed after its first sentence (consumer gone): the started generates
    and the vocoder call complete in the generator's cleanup, and the engine serves
    the next stream exactly."""
    from genie_tts_amd.inference import GENIE, ReferenceAudio
    m, _ = model
    ref = ReferenceAudio(phonemes_seq=synth.synth_phones(12, "c-r"), text_bert=np.zeros((12, 1024), np.float32),
                         audio_32k=synth.synth_ref_audio(32000 * 2, "c-a").reshape(1, -1),
                         ssl_content=synth.synth_ssl(41, "c-s").reshape(1, 768, -1))
    texts = [synth.synth_phones(n, f"c-t{n}") for n in (11, 14, 9, 16)]
    gen = GENIE()
    sp = m.T2S_FIRST_STAGE_DECODER.sampler
    args = (ref, m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER, m.VITS, None)
    try:
        it = gen.tts_stream(texts, *args, sampler=sp, vocoder_cus=64)
        first = next(it)
        it.close()
        assert not getattr(m.ENGINE, "_gq", None)
        again = list(gen.tts_stream(texts, *args, sampler=sp, vocoder_cus=64))
    finally:
        m.ENGINE.set_vocoder_cus(0)
    np.testing.assert_allclose(first, again[0], atol=1e-6)
    for t, a in zip(texts, again):
        np.testing.assert_allclose(gen.tts(t, *args, sampler=sp), a, atol=1e-6)
