"""Run the reference graph templates through the numpy executor (oracle tooling).

TEST INFRASTRUCTURE ONLY.  Needs `/root/reference` (present only in the build
container), so it is used by `tests/golden/make_golden.py` to produce the
committed golden fixtures, and by CPU tests that skip when the reference tree
is absent.  Mirrors the call sites `g/Core/Inference.py:76,88,102,47,55` and
`g/Audio/ReferenceAudio.py:73`.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Optional

import numpy as np

from .onnx_interp import Interpreter
from .onnx_wire import load_model

REF_DATA = os.environ.get("GENIE_REF_DATA", "/root/reference/src/genie_tts/Data")

_CACHE: Dict[str, object] = {}


def available() -> bool:
    return os.path.isdir(REF_DATA)


def graph(rel: str):
    if rel not in _CACHE:
        _CACHE[rel] = load_model(os.path.join(REF_DATA, rel))
    return _CACHE[rel]


def _f32(w: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    return {k: np.asarray(v, dtype=np.float32) for k, v in w.items()}


def ones_like(x, a):
    return np.ones_like(x, dtype=np.float32)


def zeros_like(x, a):
    return np.zeros_like(x, dtype=np.float32)


def t2s_encoder(w, ref_seq, text_seq, ref_bert, text_bert, ssl_content):
    it = Interpreter(graph("v2/Models/t2s_encoder_fp32.onnx"), _f32(w))
    return it.run(dict(ref_seq=ref_seq, text_seq=text_seq, ref_bert=ref_bert,
                       text_bert=text_bert, ssl_content=ssl_content))


def t2s_first_stage(w, x, prompts, noise: Callable = ones_like, trace=None):
    it = Interpreter(graph("v2/Models/t2s_first_stage_decoder_fp32.onnx"), _f32(w),
                     random_normal=noise, trace=trace)
    return it.run(dict(x=x, prompts=prompts))


def t2s_stage(w, y, y_emb, kv, noise: Callable = ones_like, trace=None):
    g = graph("v2/Models/t2s_stage_decoder_fp32.onnx")
    it = Interpreter(g, _f32(w), random_normal=noise, trace=trace)
    names = [i[0] for i in g.inputs]
    feeds = {n: v for n, v in zip(names, [y, y_emb, *kv])}
    return it.run(feeds)


def t2s_cpu(w_enc, w_t2s, ref_seq, ref_bert, text_seq, text_bert, ssl_content,
            noise: Callable = ones_like, max_steps: int = 500, force_steps: Optional[int] = None):
    """The loop of `g/Core/Inference.py:63-109` over the graphs, with its trim.

    `force_steps` ignores the stop flag for exactly that many steps (timing /
    random-weight configs where EOS never fires); None = reference behaviour.
    Returns (pred_semantic [1,1,n], per-step stop flags, first-stage y).
    """
    x, prompts = t2s_encoder(w_enc, ref_seq, text_seq, ref_bert, text_bert, ssl_content)
    y, y_emb, *kv = t2s_first_stage(w_t2s, x, prompts, noise)
    y0 = y.copy()
    stops = []
    idx = 0
    n_iter = max_steps if force_steps is None else force_steps
    for idx in range(0, n_iter):
        y, y_emb, stop, *kv = t2s_stage(w_t2s, y, y_emb, kv, noise)
        stops.append(bool(stop))
        if force_steps is None and stop:
            break
    y = y.copy()
    y[0, -1] = 0
    return np.expand_dims(y[:, -idx:], axis=0), stops, y0, x, prompts


def eos_filter(semantic_tokens: np.ndarray) -> np.ndarray:
    """`g/Core/Inference.py:41-44`."""
    eos_indices = np.where(semantic_tokens >= 1024)
    if len(eos_indices[0]) > 0:
        first_eos_index = eos_indices[-1][0]
        semantic_tokens = semantic_tokens[..., :first_eos_index]
    return semantic_tokens


def vits(version: str, w, text_seq, pred_semantic, ref_audio=None, ge=None, ge_advanced=None,
         noise: Callable = zeros_like, trace=None, fetch=None):
    rel = "v2/Models/vits_fp32.onnx" if version == "v2" else "v2ProPlus/Models/vits_fp32.onnx"
    it = Interpreter(graph(rel), _f32(w), random_normal=noise, trace=trace)
    feeds = dict(text_seq=text_seq, pred_semantic=pred_semantic)
    if version == "v2":
        feeds["ref_audio"] = ref_audio
    else:
        feeds["ge"] = ge
        feeds["ge_advanced"] = ge_advanced
    return it.run(feeds, fetch)


def prompt_encoder(w, ref_audio, sv_emb, trace=None):
    it = Interpreter(graph("v2ProPlus/Models/prompt_encoder_fp32.onnx"), _f32(w), trace=trace)
    return it.run(dict(ref_audio=ref_audio, sv_emb=sv_emb))
