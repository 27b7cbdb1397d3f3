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
  configs[3] mixed100()      V2ProPlus EN+ZH 100-sentence set, S~U[20,60],
                             G~U[50,110]; EN BERT zeros, ZH BERT from RoBERTa
                             (GetPhonesAndBert.py:64-74) over each ZH sentence's
                             synthetic token ids + word2ph (Item.bert_ids/word2ph),
                             computed by the engine (gsv_roberta_batch) in the
                             bench's timed region, by oracle/bert.py for fixtures
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
    bert_ids: Optional[np.ndarray] = None   # ZH: RoBERTa input_ids [C + 2] (CLS .. SEP)
    word2ph: Optional[np.ndarray] = None    # ZH: phones per character [C], sum = S

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


CLS_ID, SEP_ID = 101, 102


def zh_tokens(S: int, tag: str):
    """RoBERTa inputs of a synthetic Chinese sentence of S phones (the '。' prefix is one
    character of one phone, every other character two phones -- initial + final, as
    chinese_to_phones emits them; an odd count ends on a one-phone character):
    input_ids [C + 2] = CLS, C vocabulary ids, SEP and word2ph [C], sum(word2ph) = S."""
    w2p = [1] + [2] * ((S - 1) // 2) + ([1] if (S - 1) % 2 else [])
    r = synth.rng_for("zh-ids:" + tag)
    ids = np.concatenate([[CLS_ID], r.integers(672, 8000, size=len(w2p)), [SEP_ID]]).astype(np.int64)
    return ids, np.asarray(w2p, np.int64)


def mixed100(n: int = 100, tag: str = "m100") -> Workload:
    """configs[3]: V2ProPlus EN+ZH sentences (alternating); EN BERT zeros, ZH BERT from
    RoBERTa over the sentence's input_ids / word2ph (text_bert left None here)."""
    r = synth.rng_for("workload:" + tag)
    S = r.integers(20, 61, size=n)
    G = r.integers(50, 111, size=n)
    items = []
    for i in range(n):
        lang = "zh" if i % 2 == 0 else "en"
        ts = synth.synth_phones(int(S[i]), f"{tag}-t{i}", lang=lang)
        ids, w2p = zh_tokens(int(S[i]), f"{tag}-{i}") if lang == "zh" else (None, None)
        items.append(Item(ts, None, int(G[i]) + 1, lang, ids, w2p))
    return Workload(f"configs[3] mixed{n}", "v2ProPlus", reference(tag, sv=True), items)


def roberta_weights(n_layers: int = 24):
    """Synthetic RoBERTa (chinese-roberta-wwm-ext-large shapes) for the ZH sentences,
    fp32-valued: the reference loads RoBERTa.onnx with its fp32 initializers
    (ModelManager.py:139-142), with no fp16 bin."""
    from . import weights as W
    return synth.synth_weights(W.roberta_spec(n_layers), fp16=False)
