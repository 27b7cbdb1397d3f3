"""Shared fixtures for parity tests: synthetic characters and inputs."""
from __future__ import annotations

import functools

import numpy as np

from genie_tts_amd import synth, weights as W


@functools.lru_cache(maxsize=4)
def character(version: str = "v2"):
    return synth.synthetic_character(version)


def t2s_inputs(R=12, S=10, H=41, tag="a", bert=False):
    ref = synth.synth_phones(R, "r" + tag)
    txt = synth.synth_phones(S, "t" + tag)
    if bert:
        rb = synth.rng_for("rb" + tag).standard_normal((R, 1024)).astype(np.float32)
        tb = synth.rng_for("tb" + tag).standard_normal((S, 1024)).astype(np.float32)
    else:
        rb = np.zeros((R, 1024), np.float32)
        tb = np.zeros((S, 1024), np.float32)
    ssl = synth.synth_ssl(H, "s" + tag)
    return ref, txt, rb, tb, ssl


def div_term_f32():
    import math
    return np.exp(np.arange(0, 512, 2, dtype=np.float32) * np.float32(-(math.log(10000.0) / 512)))
