#!/usr/bin/env python3
"""Generate tests/golden/t2s_mixed100.npz: the configs[3] workload (V2ProPlus EN+ZH
100-sentence set, S~U[20,60], forced G~U[50,110]; genie_tts_amd.workloads.mixed100)
through the CPU oracle, greedy (RandomNormalLike := 1):

  ZH sentences: text_bert = RoBERTa features of the sentence's input_ids / word2ph
                (GetPhonesAndBert.py:64-74) from oracle/bert.py (transformers
                BertModel, hidden_states[-3], rows repeated by word2ph) on the
                synthetic 24-layer RoBERTa weights (workloads.roberta_weights);
  EN sentences: text_bert = zeros (GetPhonesAndBert.py:58-60);
  then oracle/restate.py's T2S loop (Inference.py:63-109, trim + EOS filter
  Inference.py:41-44,108-109) per sentence with the V2ProPlus character's T2S.

Fixture = lengths + output token ids + a checksum row of each ZH sentence's BERT
features (data only).  Runs ~2 min on 8 cores.
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

_CACHE = {}


def _model():
    if "m" not in _CACHE:
        from genie_tts_amd import synth
        from oracle import restate as R
        w = synth.synthetic_character("v2ProPlus")
        _CACHE["w"], _CACHE["m"] = w, R.T2SModel(w["t2s"])
    return _CACHE["w"], _CACHE["m"]


def _job(args):
    b, text_bert = args
    import torch
    torch.set_num_threads(1)
    from genie_tts_amd import workloads
    from oracle import restate as R
    w, m = _model()
    wl = workloads.mixed100()
    it, ref = wl.items[b], wl.reference
    tb = np.zeros((it.text_seq.shape[1], 1024), np.float32) if text_bert is None else text_bert
    sem, _, _ = R.t2s_generate(w["t2s_encoder"], m, ref.ref_seq, ref.ref_bert, it.text_seq, tb, ref.ssl,
                               force_steps=it.force_steps)
    return b, np.asarray(sem).reshape(-1)


def zh_berts(wl):
    from genie_tts_amd import workloads
    from oracle import bert as B
    bm = B.bert_model(workloads.roberta_weights(), 24)
    return {i: B.bert_features(bm, it.bert_ids, it.word2ph) for i, it in enumerate(wl.items) if it.bert_ids is not None}


def main():
    from genie_tts_amd import workloads
    wl = workloads.mixed100()
    n = len(wl.items)
    bert = zh_berts(wl)
    G = np.array([it.tokens for it in wl.items], np.int32)
    S = np.array([it.text_seq.shape[1] for it in wl.items], np.int32)
    out = np.full((n, G.max()), -1, np.int16)
    lens = np.zeros(n, np.int32)
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for b, tok in ex.map(_job, [(b, bert.get(b)) for b in range(n)]):
            out[b, :tok.size] = tok
            lens[b] = tok.size
    zh = np.array(sorted(bert), np.int32)
    bert_sum = np.stack([bert[i].sum(axis=0, dtype=np.float64) for i in zh]).astype(np.float32)   # [n_zh, 1024]
    np.savez_compressed(os.path.join(HERE, "t2s_mixed100.npz"), S=S, G=G, greedy=out, greedy_len=lens,
                        zh=zh, bert_colsum=bert_sum)
    print("lens", lens.tolist())


if __name__ == "__main__":
    main()
