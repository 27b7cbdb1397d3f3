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

Input normalisation.  GPT-SoVITS's CNHubert module wraps HubertModel with a
Wav2Vec2FeatureExtractor (zero-mean / unit-variance per clip when do_normalize),
but its inference path calls the inner model directly on the raw 16 kHz clip
(`ssl_model.model(wav16k.unsqueeze(0))["last_hidden_state"]` in GPT-SoVITS's
inference_webui.get_tts_wav), and Genie feeds `cn_hubert.run({'input_values':
audio_16k})` with the raw clip (ReferenceAudio.py:48-52).  So the graph's input is
raw audio and the oracle's default is `normalize=False`; `normalize=True` is the
CNHubert.forward variant, kept so tests can show the choice matters (the two differ
far beyond the parity tolerance) -- whether the absent chinese-hubert-base.onnx bakes
that step in stays unpinned.
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


def feature_normalize(audio_16k: np.ndarray) -> np.ndarray:
    """Wav2Vec2FeatureExtractor(do_normalize=True): (x - mean) / sqrt(var + 1e-7) per clip."""
    x = np.asarray(audio_16k, np.float32).reshape(-1)
    return ((x - x.mean()) / np.sqrt(x.var() + 1e-7)).astype(np.float32)


@torch.no_grad()
def ssl_content(model, audio_16k: np.ndarray, normalize: bool = False) -> np.ndarray:
    """[1, 768, T] = HubertModel(audio)["last_hidden_state"].transpose(1, 2); normalize=True
    first applies CNHubert.forward's feature-extractor normalisation (see the module doc)."""
    a = feature_normalize(audio_16k) if normalize else np.asarray(audio_16k, np.float32)
    x = torch.from_numpy(a.reshape(1, -1))
    return model(x).last_hidden_state.transpose(1, 2).numpy()
