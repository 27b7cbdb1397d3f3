"""Deterministic synthetic weights and inputs (no checkpoints exist offline).

Every tensor is a pure function of (seed, tensor name, element index):
    h   = fnv1a64(name) ^ seed
    z_i = splitmix64(h + (i + 1) * 0x9E3779B97F4A7C15)
    u_i = (z_i >> 40) / 2^24            in [0, 1)
then scaled per tensor role and rounded to fp16 (the Genie bins are fp16,
`g/ModelManager.py:75-76`; `t2s_encoder_fp32.bin` stays fp32).  The scheme is
reproducible bit-for-bit from C/Python/numpy on any box.  Scales keep
activations O(1) through 24 post-norm layers and the vocoder so that parity
tests exercise realistic magnitudes.
"""
from __future__ import annotations

import re
from typing import Dict, Optional, Tuple

import numpy as np

from . import weights as W

WEIGHT_SEED = 0x6E1E
INPUT_SEED = 20260116

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for c in s.encode():
        h ^= c
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def uniform01(name: str, n: int, seed: int = WEIGHT_SEED) -> np.ndarray:
    """u_i in [0,1) as float64, exactly representable (24-bit mantissa)."""
    h = np.uint64((fnv1a64(name) ^ seed) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = h + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)


def _role_scale(name: str, shape: Tuple[int, ...]) -> Tuple[float, float]:
    """(center, half-width) of the uniform distribution for this tensor."""
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "alpha":
        return 1.0, 0.2
    if leaf in ("gamma",) or re.search(r"(norm\d?|LayerNorm)\.weight$", name):
        return 1.0, 0.1
    if leaf in ("beta",) or re.search(r"(norm\d?|LayerNorm)\.bias$", name):
        return 0.0, 0.05
    if leaf == "weight_g":
        return 1.0, 0.25
    if leaf == "bias" or leaf.endswith("_bias"):
        return 0.0, 0.05
    if leaf == "prelu" or name.endswith("prelu.weight"):
        return 0.25, 0.05
    if "emb_rel" in leaf:
        return 0.0, 0.3
    if ("embed" in name or "embedding" in name) and "pos_conv_embed" not in name:
        return 0.0, 1.0
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        if name.endswith("weight_v"):
            return 0.0, 1.0          # direction only; weight_g sets the norm
        return 0.0, float(np.sqrt(3.0 / fan_in))
    return 0.0, 0.1


def synth_tensor(name: str, shape: Tuple[int, ...], seed: int = WEIGHT_SEED,
                 fp16: bool = True) -> np.ndarray:
    n = int(np.prod(shape))
    c, w = _role_scale(name, shape)
    v = (c + w * (2.0 * uniform01(name, n, seed) - 1.0)).reshape(shape)
    return v.astype(np.float16) if fp16 else v.astype(np.float32)


def synth_weights(spec, seed: int = WEIGHT_SEED, fp16: bool = True) -> Dict[str, np.ndarray]:
    return {k: synth_tensor(k, s, seed, fp16) for k, s in spec.items()}


def synth_sv_weights(seed: int = WEIGHT_SEED) -> Dict[str, np.ndarray]:
    """fp32 weights for the SV model (weights.sv_spec): convs uniform with variance
    1/fan_in; BatchNorm weight 1 +- 0.2, bias and running_mean +- 0.1, running_var
    in [0.5, 1.5] (the real speaker_encoder.onnx ships fp32, so nothing is rounded)."""
    out = {}
    for name, shape in W.sv_spec().items():
        n = int(np.prod(shape))
        u = 2.0 * uniform01(name, n, seed) - 1.0
        leaf = name.rsplit(".", 1)[-1]
        if len(shape) == 4:
            v = u * np.sqrt(3.0 / int(np.prod(shape[1:])))
        elif leaf == "running_var":
            v = 1.0 + 0.5 * u
        elif leaf == "weight":
            v = 1.0 + 0.2 * u
        else:
            v = 0.1 * u
        out[name] = v.reshape(shape).astype(np.float32)
    return out


def synthetic_character(version: str = "v2", seed: int = WEIGHT_SEED):
    """Weights of a synthetic character in the same form `load_character_weights` returns."""
    w = {
        "t2s_encoder": synth_weights(W.t2s_encoder_spec(), seed, fp16=False),
        "t2s": synth_weights(W.t2s_spec(), seed),
        "vits": synth_weights(W.vits_spec(version), seed),
    }
    if version != "v2":
        w["prompt_encoder"] = synth_weights(W.prompt_encoder_spec(), seed)
    return w


# ------------------------------------------------------------------- inputs
# Japanese phone ids of symbols_v2 (g/G2P/SymbolsV2.py): the 38 JP phones
# plus prosody marks and punctuation; '.' is the '。' prefix token.
JP_PHONE_IDS = (
    52, 64, 82, 96, 122, 123, 125, 126, 127, 128, 129, 155, 156, 157, 158,
    159, 160, 221, 222, 223, 225, 226, 227, 228, 229, 245, 246, 248, 249,
    250, 251, 252, 253, 254, 295, 316, 318, 319,   # JAPANESE_SYMBOLS
    322, 323, 95, 1, 3,                            # '[' ']' '_' ',' '.'
)
DOT_ID = 3
# English (ARPAbet) and Chinese (pinyin initials + toned finals) phone ids of the
# same table (g/G2P/SymbolsV2.py: symbol_to_id_v2 over ARPABET_SYMBOLS and
# PINYIN_INITIALS / PINYIN_FINALS_BASE x tones 1-5), for the EN+ZH workload.
EN_PHONE_IDS = tuple(list(range(6, 28)) + list(range(34, 44)) + [49, 50, 51] + list(range(53, 66)) +
                     list(range(67, 77)) + [80, 81] + list(range(83, 86)) + list(range(87, 95)))
ZH_PHONE_IDS = tuple([5] + list(range(28, 34)) + list(range(44, 49)) + [66] + list(range(97, 123)) +
                     [124, 125, 127] + list(range(130, 157)) + [158] + list(range(161, 223)) +
                     [224, 225, 227] + list(range(230, 246)) + [247, 248, 250, 251, 252] +
                     list(range(255, 295)) + list(range(296, 321)))


def rng_for(tag: str, seed: int = INPUT_SEED) -> np.random.Generator:
    return np.random.default_rng([seed, fnv1a64(tag) & 0xFFFFFFFF])


def synth_phones(n: int, tag: str, seed: int = INPUT_SEED, lang: str = "ja") -> np.ndarray:
    r = rng_for("phones:" + tag, seed)
    table = {"ja": JP_PHONE_IDS, "en": EN_PHONE_IDS, "zh": ZH_PHONE_IDS}[lang]
    ids = r.choice(np.array(table, dtype=np.int64), size=n)
    ids[0] = DOT_ID
    return ids.reshape(1, n)


def synth_ssl(h: int, tag: str = "ref", seed: int = INPUT_SEED) -> np.ndarray:
    return rng_for("ssl:" + tag, seed).standard_normal((1, 768, h)).astype(np.float32)


def synth_ref_audio(n32: int, tag: str = "ref", seed: int = INPUT_SEED) -> np.ndarray:
    return (0.1 * rng_for("audio:" + tag, seed).standard_normal((1, n32))).astype(np.float32)


def synth_ge(dim: int, tag: str = "ge", seed: int = INPUT_SEED) -> np.ndarray:
    return rng_for("ge:" + tag, seed).standard_normal((1, dim, 1)).astype(np.float32)
