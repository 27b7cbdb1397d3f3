"""Deterministic stand-ins for benchmarks and tests: a G2P (outside the engine, SURVEY
§8: out of scope) and SSL features in place of a real clip's CN-HuBERT output (the
engine runs CN-HuBERT itself, gsv_hubert, once weights are loaded; the benchmarks and
the server's --ssl option use this stand-in instead so they need no HuBERT weights).
The product path uses them only when a caller configures them explicitly
(api.set_g2p / set_ssl_extractor, server --g2p/--ssl).

toy_g2p maps each character to two Japanese phone ids (a 20-character sentence
-> ~40 phones, the nominal S=45 of SURVEY §8 with the '。' prefix), BERT zeros
(Japanese); toy_ssl returns seeded N(0,1) features of the HuBERT frame count
(one frame per 320 samples at 16 kHz).
"""
from __future__ import annotations

import numpy as np

from . import synth


def toy_g2p(text: str, language: str = "Japanese"):
    ids = []
    for c in text:
        if c in "。.":
            ids.append(synth.DOT_ID)
        else:
            o = ord(c)
            ids += [synth.JP_PHONE_IDS[o % len(synth.JP_PHONE_IDS)], synth.JP_PHONE_IDS[(o // 7) % 38]]
    return np.asarray(ids, np.int64).reshape(1, -1), np.zeros((len(ids), 1024), np.float32)


def toy_ssl(audio_16k) -> np.ndarray:
    n = np.asarray(audio_16k).shape[-1] // 320
    return synth.rng_for(f"toy-ssl-{n}").standard_normal((1, 768, n)).astype(np.float32)
