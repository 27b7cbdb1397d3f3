"""Synthetic workloads of BASELINE.json's configs, shared by
bench.py, the golden-fixture generators and the tests.

No G2P, HuBERT or checkpoints exist offline, so every workload is seeded
synthetic phone ids / features of the nominal shapes ("Nominal
shapes"): reference R=48 phones, H=264 HuBERT frames (P=132 prompts), 5.3 s
of 32 kHz reference audio.  Random weights never emit EOS, so each utterance
runs a forced number of loop steps: `force_steps` = G + 1 loop steps keep G
semantic tokens (the trim of Inference.py:108-109 drops the last one).

  configs[1] single()        one 20-char JP utterance, S=45, G=80
  configs[2] batch64()       64 mixed-length JP sentences, S~U[30,60], G~U[50,110]
  configs[3] mixed100()      V2ProPlus EN+ZH 100-sentence set (ZH BERT ~ N(0,1)
                             as a RoBERTa stand-in, EN BERT zeros), S~U[20,60],
                             G~U[50,110]
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import synth

R_PH, S_PH, H_SSL = 48, 45, 264
REF_AUDIO_S = 5.3
SR = 32000
NOMINAL_G = 80


@dataclass
class Reference:
    """Features of one reference clip (ReferenceAudio.py:28-76)."""
    ref_seq: np.ndarray                  # i64 [1, R]
    ref_bert: np.ndarray                 # f32 [R, 1024]
    ssl: np.ndarray                      # f32 [1, 768, H]
    audio_32k: np.ndarray                # f32 [1, N32]
    sv_emb: Optional[np.ndarray] = None  # f32 [1, 20480] (V2ProPlus)


@dataclass
class Item:
    """One sentence of a workload."""
    text_seq: np.ndarray                 # i64 [1, S]
    text_bert: Optional[np.ndarray]      # f32 [S, 1024] or None (zeros)
    force_steps: int                     # loop steps (G + 1)
    lang: str = "ja"

    @property
    def tokens(self) -> int:
        return self.force_steps - 1


@dataclass
class Workload:
    name: str
    version: str                         # "v2" | "v2ProPlus"
    reference: Reference
    items: List[Item] = field(default_factory=list)
    top_k: int = 15
    greedy: bool = True

    @property
    def total_tokens(self) -> int:
        return sum(i.tokens for i in self.items)

    @property
    def total_samples(self) -> int:
        return 1280 * self.total_tokens


def reference(tag: str = "bench", R: int = R_PH, H: int = H_SSL, sv: bool = False) -> Reference:
    return Reference(
        ref_seq=synth.synth_phones(R, tag + "-ref"),
        ref_bert=np.zeros((R, 1024), np.float32),      # JP reference text: BERT features are zeros
        ssl=synth.synth_ssl(H, tag),
        audio_32k=synth.synth_ref_audio(int(REF_AUDIO_S * SR), tag),
        sv_emb=synth.rng_for("sv:" + tag).standard_normal((1, 20480)).astype(np.float32) if sv else None)


def single() -> Workload:
    """configs[1]: the bench's historical inputs (tags "bench-ref", "bench-text")."""
    ref = Reference(ref_seq=synth.synth_phones(R_PH, "bench-ref"), ref_bert=np.zeros((R_PH, 1024), np.float32),
                    ssl=synth.synth_ssl(H_SSL, "bench"),
                    audio_32k=synth.synth_ref_audio(int(REF_AUDIO_S * SR), "bench"))
    item = Item(synth.synth_phones(S_PH, "bench-text"), None, NOMINAL_G + 1)
    return Workload("configs[1] single", "v2", ref, [item])


def batch64(n: int = 64, tag: str = "b64") -> Workload:
    """configs[2]: n mixed-length JP sentences, S~U[30,60], G~U[50,110], top-k 5 sampled."""
    r = synth.rng_for("workload:" + tag)
    S = r.integers(30, 61, size=n)
    G = r.integers(50, 111, size=n)
    items = [Item(synth.synth_phones(int(S[i]), f"{tag}-t{i}"), None, int(G[i]) + 1) for i in range(n)]
    return Workload(f"configs[2] batch{n}", "v2", reference(tag), items, top_k=5, greedy=False)


def mixed100(n: int = 100, tag: str = "m100") -> Workload:
    """configs[3]: V2ProPlus EN+ZH sentences (alternating), ZH BERT ~ N(0,1), EN BERT zeros."""
    r = synth.rng_for("workload:" + tag)
    S = r.integers(20, 61, size=n)
    G = r.integers(50, 111, size=n)
    items = []
    for i in range(n):
        lang = "zh" if i % 2 == 0 else "en"
        ts = synth.synth_phones(int(S[i]), f"{tag}-t{i}", lang=lang)
        tb = (synth.rng_for(f"{tag}-bert{i}").standard_normal((int(S[i]), 1024)).astype(np.float32)
              if lang == "zh" else None)
        items.append(Item(ts, tb, int(G[i]) + 1, lang))
    return Workload(f"configs[3] mixed{n}", "v2ProPlus", reference(tag, sv=True), items)
