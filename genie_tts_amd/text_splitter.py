"""Sentence splitting for `tts(..., split_sentence=True)` with the semantics of
the reference's TextSplitter (src/genie_tts/Utils/TextSplitter.py:5-123), used
by its TTS worker (Core/TTSPlayer.py feed()):

- runs of punctuation form one block; a block holding any terminator
  (。！？… ! ? .) closes the sentence once its effective length reaches
  `min_len`, a block of separators only (， 、 ； ： —— , ; : and quotes) closes
  it once the effective length reaches `max_len`;
- effective length skips punctuation and counts ASCII characters 1, others 2;
- newlines are dropped; the tail is kept if it has content, otherwise glued to
  the previous sentence.
"""
from __future__ import annotations

import re
from typing import List

TERMINATORS = frozenset("。！？…!?.")
SEPARATORS = frozenset(["，", "、", "；", "：", "——", ",", ";", ":", "“", "”", "‘", "’", '"', "'"])
PUNCTUATION = TERMINATORS | SEPARATORS


class TextSplitter:
    def __init__(self, max_len: int = 40, min_len: int = 5):
        self.max_len = max_len
        self.min_len = min_len
        alts = sorted(PUNCTUATION, key=len, reverse=True)        # longest first ("——" before "—")
        self._blocks = re.compile("((?:" + "|".join(re.escape(p) for p in alts) + ")+)")

    @staticmethod
    def char_width(ch: str) -> int:
        return 1 if ord(ch) < 128 else 2

    def effective_len(self, text: str) -> int:
        return sum(self.char_width(c) for c in text if c not in PUNCTUATION)

    @staticmethod
    def closes_sentence(block: str) -> bool:
        return any(c in TERMINATORS for c in block)

    def split(self, text: str) -> List[str]:
        if not text:
            return []
        out: List[str] = []
        buf = ""
        for piece in self._blocks.split(text.replace("\n", "")):
            if not piece:
                continue
            buf += piece
            if piece[0] not in PUNCTUATION:          # plain text: keep accumulating
                continue
            limit = self.min_len if self.closes_sentence(piece) else self.max_len
            if self.effective_len(buf) >= limit:
                out.append(buf.strip())
                buf = ""
        tail = buf.strip()
        if tail:
            if self.effective_len(tail) > 0:
                out.append(tail)
            elif out:
                out[-1] += tail
        return out
