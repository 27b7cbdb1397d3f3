"""CPU: pin tests/golden/t2s_mixed100.npz to the oracle (oracle/bert.py +
oracle/restate.py) on one English and one Chinese utterance, and check the workload
definition the fixture was generated from (lengths, languages, RoBERTa inputs)."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden", "t2s_mixed100.npz")


def test_workload_shape():
    from genie_tts_amd import workloads
    g = np.load(GOLD)
    wl = workloads.mixed100()
    assert len(wl.items) == 100 and wl.version == "v2ProPlus"
    assert [it.text_seq.shape[1] for it in wl.items] == g["S"].tolist()
    assert [it.tokens for it in wl.items] == g["G"].tolist()
    zh = [i for i, it in enumerate(wl.items) if it.lang == "zh"]
    assert zh == g["zh"].tolist() and len(zh) == 50
    for it in wl.items:
        if it.lang == "zh":   # word2ph covers the phones; CLS + one id per character + SEP
            assert int(it.word2ph.sum()) == it.text_seq.shape[1]
            assert it.bert_ids.size == it.word2ph.size + 2 and it.bert_ids[0] == 101 and it.bert_ids[-1] == 102
        else:
            assert it.bert_ids is None and it.text_bert is None


def test_fixture_rows_match_oracle():
    from tests.golden.make_mixed100 import _job
    from genie_tts_amd import workloads
    from oracle import bert as B
    g = np.load(GOLD)
    wl = workloads.mixed100()
    bm = B.bert_model(workloads.roberta_weights(), 24)
    it = wl.items[0]
    bert0 = B.bert_features(bm, it.bert_ids, it.word2ph)
    np.testing.assert_allclose(bert0.sum(0, dtype=np.float64), g["bert_colsum"][0], rtol=0, atol=1e-3)
    for b, tb in ((0, bert0), (1, None)):      # ZH, EN
        _, tok = _job((b, tb))
        assert tok.tolist() == g["greedy"][b, :g["greedy_len"][b]].astype(np.int64).tolist()
