"""RoBERTa BERT-feature oracle (TEST INFRASTRUCTURE ONLY: imported by tests/).

The reference runs GenieData RoBERTa.onnx (`g/GetPhonesAndBert.py:64-74`), GPT-SoVITS's
get_bert_feature over chinese-roberta-wwm-ext-large: BertModel(input_ids,
attention_mask, output_hidden_states=True).hidden_states[-3][0][1:-1], each
character row repeated word2ph[i] times.  The graph is absent here, so the oracle
is transformers' BertModel (hidden 1024, 16 heads, FFN 4096, GELU, LayerNorm
eps 1e-12) loaded with the engine's synthetic weights
(genie_tts_amd.weights.roberta_spec names).  ONNX-level parity: UNPINNED.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def bert_model(w: Dict[str, np.ndarray], n_layers: int = 24):
    from transformers import BertConfig, BertModel
    cfg = BertConfig(vocab_size=w["embeddings.word_embeddings.weight"].shape[0], hidden_size=1024,
                     num_hidden_layers=n_layers, num_attention_heads=16, intermediate_size=4096,
                     hidden_act="gelu", max_position_embeddings=w["embeddings.position_embeddings.weight"].shape[0],
                     type_vocab_size=2, layer_norm_eps=1e-12)
    m = BertModel(cfg, add_pooling_layer=False).eval()
    sd = m.state_dict()
    new = {k: (torch.from_numpy(np.asarray(w[k], np.float32).copy()) if k in w else sd[k]) for k in sd}
    m.load_state_dict(new, strict=True)
    return m


@torch.no_grad()
def bert_features(model, input_ids: np.ndarray, word2ph: np.ndarray) -> np.ndarray:
    ids = torch.from_numpy(np.asarray(input_ids, np.int64).reshape(1, -1))
    out = model(input_ids=ids, attention_mask=torch.ones_like(ids), output_hidden_states=True)
    res = out.hidden_states[-3][0][1:-1]
    rep = torch.from_numpy(np.asarray(word2ph, np.int64))
    return torch.repeat_interleave(res[: len(rep)], rep, dim=0).numpy()
