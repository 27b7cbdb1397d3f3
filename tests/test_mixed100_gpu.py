"""configs[3] on the GPU: the V2ProPlus EN+ZH 100-sentence set through the replica
path the bench and the 8-GPU runs use -- replicas.run_sharded(requests,
engine_synth(...), rank, world) -- on the HIP engine:

  * Chinese sentences' BERT features from the engine's RoBERTa (gsv_roberta_batch,
    synthetic 24-layer chinese-roberta-wwm-ext-large weights; the reference runs
    RoBERTa per Chinese sentence, GetPhonesAndBert.py:64-74), English zeros;
  * one batched T2S per shard, vocoder lanes per utterance, V2ProPlus ge / ge_advanced
    from the engine's prompt encoder (ReferenceAudio.py:68-76, Inference.py:52-60);

against tests/golden/t2s_mixed100.npz (tests/golden/make_mixed100.py: oracle/bert.py
+ oracle/restate.py): per-utterance greedy token ids bit-exact, the RoBERTa features
(column sums) within fp32 tolerance, and the audio of a few utterances within RMS 1e-4
of the oracle vocoder (zero z_p noise)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "t2s_mixed100.npz")
RMS_TOL = 1e-4


@pytest.fixture(scope="module")
def run():
    from genie_tts_amd import replicas, synth, workloads
    from genie_tts_amd.engine import make_sampler
    from genie_tts_amd.inference import ReferenceAudio, tts_client
    from genie_tts_amd.model_manager import build_model
    w = synth.synthetic_character("v2ProPlus")
    w["roberta"] = workloads.roberta_weights()
    model = build_model(w, "v2ProPlus", "Chinese", sampler=make_sampler(greedy=True))
    model.VITS.noise = "zero"
    wl = workloads.mixed100()
    ref = wl.reference
    refa = ReferenceAudio(phonemes_seq=ref.ref_seq, text_bert=ref.ref_bert, audio_32k=ref.audio_32k,
                          ssl_content=ref.ssl, sv_emb=ref.sv_emb)
    reqs = [replicas.Request(i, it.text_seq, None, it.force_steps, it.bert_ids, it.word2ph)
            for i, it in enumerate(wl.items)]
    toks = {}
    orig = tts_client.tts_batch_t2s

    def record(items, prompt_audio, m, sampler):   # the T2S tokens, recorded on their way to the vocoder
        out = orig(items, prompt_audio, m, sampler)
        for it, t in zip(items, out):
            toks[id(it[0])] = t
        return out
    tts_client.tts_batch_t2s = record
    try:
        wavs = replicas.run_sharded(reqs, replicas.engine_synth(model, refa, lambda: make_sampler(greedy=True),
                                                                roberta=model.ENGINE), 0, 1)
    finally:
        tts_client.tts_batch_t2s = orig
    yield dict(w=w, wl=wl, refa=refa, model=model, wavs=wavs, toks=[toks[id(it.text_seq)] for it in wl.items])
    model.ENGINE.close()


def test_mixed100_tokens_bit_exact(run):
    g = np.load(GOLD)
    wl = run["wl"]
    assert [it.tokens for it in wl.items] == g["G"].tolist()
    bad = []
    for b, tok in enumerate(run["toks"]):
        ref = g["greedy"][b, :g["greedy_len"][b]].astype(np.int64)
        if tok.tolist() != ref.tolist():
            n = min(tok.size, ref.size)
            i = next((j for j in range(n) if tok[j] != ref[j]), n)
            bad.append((b, wl.items[b].lang, i))
    assert not bad, f"(utterance, language, first differing token) {bad}"
    assert [w.size for w in run["wavs"]] == [1280 * int(n) for n in g["greedy_len"]]


def test_mixed100_roberta_features(run):
    """The engine's packed RoBERTa pass vs oracle/bert.py (column sums of each ZH
    sentence's [S, 1024] features, from the fixture)."""
    g = np.load(GOLD)
    wl = run["wl"]
    zh = g["zh"].tolist()
    assert zh == [i for i, it in enumerate(wl.items) if it.lang == "zh"]
    feats = run["model"].ENGINE.roberta_batch([(wl.items[i].bert_ids, wl.items[i].word2ph) for i in zh])
    got = np.stack([f.double().sum(0).cpu().numpy() for f in feats])
    rows = np.array([[wl.items[i].text_seq.shape[1]] for i in zh], np.float64)
    err = np.abs(got - g["bert_colsum"]) / np.sqrt(rows)
    assert float(err.max()) < 1e-3, float(err.max())


@pytest.mark.parametrize("b", [0, 1, 2])       # ZH, EN, ZH
def test_mixed100_audio_vs_oracle(run, b):
    import torch
    from oracle import restate as R
    w, wl, refa = run["w"], run["wl"], run["refa"]
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ge, ga = R.prompt_encoder(w["prompt_encoder"], refa.audio_32k, refa.sv_emb)
    sem = run["toks"][b].reshape(1, 1, -1)
    want = R.VitsModel(w["vits"], "v2ProPlus")(wl.items[b].text_seq, sem, ge=ge.numpy(),
                                                ge_advanced=ga.numpy()).numpy().reshape(-1)
    got = np.asarray(run["wavs"][b], np.float32).reshape(-1)
    assert got.shape == want.shape
    rms = float(np.sqrt(np.mean((got - want) ** 2)))
    print(f"utterance {b} ({wl.items[b].lang}): rms {rms:.2e}")
    assert rms <= RMS_TOL, rms


def test_mixed100_sharded_two_ranks_cover_the_set(run):
    """The LPT plan of world 2 covers the set once, and each shard's tokens (rank-local
    batches) equal the world-1 tokens: replicas change where an utterance runs, not
    what it produces."""
    from genie_tts_amd import replicas
    from genie_tts_amd.engine import make_sampler
    from genie_tts_amd.inference import tts_client
    wl, model, refa = run["wl"], run["model"], run["refa"]
    reqs = [replicas.Request(i, it.text_seq, None, it.force_steps, it.bert_ids, it.word2ph)
            for i, it in enumerate(wl.items)]
    shards = replicas.lpt_assign([replicas.predicted_cost(r) for r in reqs], 2)
    assert sorted(sum(shards, [])) == list(range(len(reqs)))
    mine = [reqs[i] for i in shards[1]]
    bert = replicas.text_berts(mine, model.ENGINE)
    toks = tts_client.tts_batch_t2s([(r.text_seq, b, r.force_steps) for r, b in zip(mine, bert)], refa, model,
                                    make_sampler(greedy=True))
    for r, t in zip(mine, toks):
        assert t.tolist() == run["toks"][r.idx].tolist(), r.idx
