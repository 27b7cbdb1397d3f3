"""CN-HuBERT oracle (TEST INFRASTRUCTURE ONLY: imported by tests/ and nothing else).

The reference runs chinese-hubert-base.onnx (`g/Audio/ReferenceAudio.py:48-52`,
`g/ModelManager.py:172-195`), an export of transformers' HubertModel that
GPT-SoVITS makes as HubertModel(raw 16 kHz audio)["last_hidden_state"]
.transpose(1, 2).  The graph and its weights are not in this container, so the
oracle is the published model itself: transformers.HubertModel (the version
installed here, `hubert_version()`), configured as chinese-hubert-base
(conv_bias=False, feat_extract_norm="group", 12 x 768, 12 heads, FFN 3072,
GELU, post-norm encoder), loaded with the engine's synthetic weights
(genie_tts_amd.weights.hubert_spec names).  ONNX-level parity: UNPINNED (no
graph file, no fixtures in the reference).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def hubert_version() -> str:
    import transformers
    return transformers.__version__


def hubert_model(w: Dict[str, np.ndarray]):
    """transformers.HubertModel (eval, fp32) holding the weights `w`."""
    from transformers import HubertConfig, HubertModel
    cfg = HubertConfig(conv_bias=False, feat_extract_norm="group", do_stable_layer_norm=False,
                       hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                       hidden_act="gelu", feat_extract_activation="gelu", layer_norm_eps=1e-5)
    m = HubertModel(cfg).eval()
    sd = m.state_dict()
    new = {}
    for k in sd:
        if "pos_conv_embed.conv.parametrizations.weight.original" in k or k.endswith("weight_g") or \
                k.endswith("weight_v"):
            continue
        if k == "masked_spec_embed":
            new[k] = sd[k]
            continue
        new[k] = torch.from_numpy(np.asarray(w[k], np.float32).copy())
    # weight norm (dim=2) with v = W and g = ||W|| per tap reproduces W
    Wp = torch.from_numpy(np.asarray(w["encoder.pos_conv_embed.conv.weight"], np.float32).copy())
    g = torch.linalg.vector_norm(Wp, dim=(0, 1), keepdim=True)
    keys = [k for k in sd if "pos_conv_embed.conv" in k and k != "encoder.pos_conv_embed.conv.bias"]
    for k in keys:
        if k.endswith("original0") or k.endswith("weight_g"):
            new[k] = g
        else:
            new[k] = Wp
    m.load_state_dict(new, strict=True)
    return m


@torch.no_grad()
def ssl_content(model, audio_16k: np.ndarray) -> np.ndarray:
    """[1, 768, T] = HubertModel(audio)["last_hidden_state"].transpose(1, 2)."""
    x = torch.from_numpy(np.asarray(audio_16k, np.float32).reshape(1, -1))
    return model(x).last_hidden_state.transpose(1, 2).numpy()
