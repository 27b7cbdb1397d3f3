"""GPU: RoBERTa BERT features on the engine (gsv_roberta, bert.hip) against the
oracle, transformers' BertModel (the published chinese-roberta-wwm-ext-large
architecture GPT-SoVITS exports) on the same synthetic weights:
hidden_states[-3], CLS/SEP dropped, rows repeated by word2ph
(GetPhonesAndBert.py:64-74).  The weights are fp32-valued like RoBERTa.onnx's
initializers, so the engine runs its split-weight GEMMs (W16 hi + lo planes).
ONNX-level parity unpinned (RoBERTa.onnx absent)."""
import numpy as np
import pytest

from genie_tts_amd import synth, weights as W

pytestmark = pytest.mark.gpu
RMS_TOL = 1e-4


def _setup(n_layers, fp16=False):
    """fp32-valued weights by default, as RoBERTa.onnx ships (ModelManager.py:139-142)."""
    from genie_tts_amd.engine import Engine
    from oracle import bert as B
    w = synth.synth_weights(W.roberta_spec(n_layers), fp16=fp16)
    e = Engine({"roberta": w}, "v2")
    # every projection of the layers that run (0 .. L-3) is an fp32 tensor -> hi + lo planes
    assert e.counter("w16_split_tensors") == (0 if fp16 else 4 * (n_layers - 2))
    return e, B, B.bert_model(w, n_layers)


@pytest.mark.parametrize("n_layers,n_chars", [(4, 9), (24, 20)])   # reduced; the real 24-layer model
def test_roberta_vs_transformers(n_layers, n_chars):
    e, B, m = _setup(n_layers)
    try:
        r = synth.rng_for(f"rb-{n_layers}")
        ids = np.concatenate([[101], r.integers(672, 8000, size=n_chars), [102]]).astype(np.int64)
        word2ph = r.integers(1, 4, size=n_chars).astype(np.int64)
        got = e.roberta(ids, word2ph, np.ones_like(ids)).cpu().numpy()
        ref = B.bert_features(m, ids, word2ph)
        assert got.shape == ref.shape == (int(word2ph.sum()), 1024)
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"layers={n_layers} rms {rms:.2e} max {np.abs(got - ref).max():.2e} std {ref.std():.3f}")
        assert rms <= RMS_TOL * max(1.0, float(ref.std())), rms
    finally:
        e.close()


def test_roberta_session_feeds_chinese_text_features():
    """A G2P returning (phones, None, input_ids, word2ph) gets its BERT rows from the engine."""
    import genie_tts_amd as genie
    from genie_tts_amd import api
    from genie_tts_amd.model_manager import model_manager
    from genie_tts_amd.sessions import RobertaSession
    e, B, m = _setup(4)
    ids = np.array([101, 1000, 2000, 3000, 102], np.int64)
    w2p = np.array([2, 1, 3], np.int64)
    phones = np.arange(6, dtype=np.int64).reshape(1, -1) + 30
    genie.set_g2p(lambda text, lang: (phones, None, ids, w2p))
    model_manager.roberta = RobertaSession(e)
    try:
        ps, tb = api._text_features("你好吗", "Chinese")
        assert tb.shape == (6, 1024)
        np.testing.assert_allclose(tb, B.bert_features(m, ids, w2p), atol=1e-4)
    finally:
        model_manager.roberta = None
        genie.set_g2p(None)
        e.close()


def test_roberta_batch_equals_single_calls():
    """gsv_roberta_batch (packed rows, per-sentence attention) returns exactly what one
    gsv_roberta call per sentence returns."""
    from genie_tts_amd import workloads
    e, B, m = _setup(4)
    try:
        sents = [workloads.zh_tokens(S, f"rbb-{S}") for S in (21, 37, 60, 8)]
        got = e.roberta_batch(sents)
        for (ids, w2p), g in zip(sents, got):
            one = e.roberta(ids, w2p).cpu().numpy()
            assert g.shape == one.shape == (int(w2p.sum()), 1024)
            assert np.array_equal(g.cpu().numpy(), one)
        ref = B.bert_features(m, sents[1][0], sents[1][1])
        assert float(np.sqrt(np.mean((got[1].cpu().numpy() - ref) ** 2))) <= RMS_TOL
    finally:
        e.close()


@pytest.mark.parametrize("fp16", [True, False])
def test_roberta_weight_precision(fp16):
    """fp16-valued weights take one plane; fp32 ones keep their low bits: rounding the
    fp32 weights to fp16 (what the engine did before) moves the output measurably more
    than the split path's error against the fp32 oracle."""
    e, B, m = _setup(4, fp16)
    try:
        r = synth.rng_for("rb-prec")
        ids = np.concatenate([[101], r.integers(672, 8000, size=12), [102]]).astype(np.int64)
        w2p = np.ones(12, np.int64)
        got = e.roberta(ids, w2p).cpu().numpy()
        ref = B.bert_features(m, ids, w2p)
        rms = float(np.sqrt(np.mean((got - ref) ** 2)))
        print(f"fp16={fp16}: rms {rms:.2e}")
        assert rms <= 5e-6 * max(1.0, float(ref.std())), rms
        if not fp16:
            w16 = {k: v.astype(np.float16).astype(np.float32)
                   for k, v in synth.synth_weights(W.roberta_spec(4), fp16=False).items()}
            rounded = B.bert_features(B.bert_model(w16, 4), ids, w2p)
            gap = float(np.sqrt(np.mean((rounded - ref) ** 2)))
            print(f"fp16-rounded weights: rms {gap:.2e}")
            assert gap > 10 * rms, (gap, rms)
    finally:
        e.close()
