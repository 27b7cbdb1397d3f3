"""The `genie_tts` entry points this engine serves (src/genie_tts/__init__.py:1-28,
src/genie_tts/Internal.py:94-310), restricted to the synthesis hot path.

Same names and argument meaning as the reference; differences, all outside the
path: reference features are supplied, not extracted from a wav
(`set_reference_audio` takes the arrays; CN-HuBERT/SV/resampling are §8(f)),
text needs a G2P callable (`set_g2p`, e.g. the reference's
`get_phones_and_bert`) or phoneme ids, and there is no playback thread: `tts`
returns the audio and optionally writes the same 16-bit mono WAV the reference's
TTSPlayer writes (TTSPlayer.py:51-53,149-158).
"""
from __future__ import annotations

import os
import wave
from typing import Callable, Dict, Optional, Sequence, Union

import numpy as np

from .inference import ReferenceAudio, tts_client
from .model_manager import model_manager

SAMPLE_RATE = 32000
_reference_audios: Dict[str, ReferenceAudio] = {}
_g2p: Optional[Callable] = None


def _norm_language(language: Optional[str]) -> str:
    if language is None:
        return "Japanese"
    l = language.lower()
    return {"ja": "Japanese", "jp": "Japanese", "japanese": "Japanese", "en": "English", "english": "English",
            "zh": "Chinese", "chinese": "Chinese", "hybrid": "Hybrid-Chinese-English",
            "hybrid-chinese-english": "Hybrid-Chinese-English"}.get(l, language)


def set_g2p(fn: Callable) -> None:
    """fn(text, language) -> (text_seq i64 [1,S], text_bert f32 [S,1024])."""
    global _g2p
    _g2p = fn


def load_character(character_name: str, onnx_model_dir: Union[str, os.PathLike], language: str) -> None:
    """Internal.py:94-126: load a converted character directory."""
    language = _norm_language(language)
    if language not in ("Japanese", "English", "Chinese", "Hybrid-Chinese-English"):
        raise ValueError("Unknown language")
    model_manager.load_character(character_name, os.fspath(onnx_model_dir), language)


def load_weights(character_name: str, weights, version: str, language: str = "Japanese") -> None:
    """Register a character from in-memory weights (e.g. genie_tts_amd.synth)."""
    model_manager.load_weights(character_name, weights, version, _norm_language(language))


def unload_character(character_name: str) -> None:
    model_manager.remove_character(character_name)


def set_reference_audio(character_name: str, phonemes_seq: np.ndarray, text_bert: Optional[np.ndarray],
                        audio_32k: np.ndarray, ssl_content: np.ndarray, sv_emb: Optional[np.ndarray] = None,
                        audio_text: str = "") -> None:
    """Internal.py:143-190 with the features the reference's ReferenceAudio computes."""
    ps = np.asarray(phonemes_seq, np.int64).reshape(1, -1)
    tb = np.zeros((ps.shape[1], 1024), np.float32) if text_bert is None else np.asarray(text_bert, np.float32)
    _reference_audios[character_name] = ReferenceAudio(
        phonemes_seq=ps, text_bert=tb, audio_32k=np.asarray(audio_32k, np.float32).reshape(1, -1),
        ssl_content=np.asarray(ssl_content, np.float32).reshape(1, 768, -1),
        sv_emb=None if sv_emb is None else np.asarray(sv_emb, np.float32).reshape(1, -1), text=audio_text)


def clear_reference_audio_cache() -> None:
    _reference_audios.clear()


def _write_wav(path: str, audio: np.ndarray) -> None:
    parent = os.path.dirname(path)
    if parent:
        os.makedirs(parent, exist_ok=True)
    with wave.open(path, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(SAMPLE_RATE)
        wf.writeframes((audio.squeeze() * 32767).astype(np.int16).tobytes())


def tts(character_name: str, text: Union[str, Sequence[int], np.ndarray], play: bool = False,
        split_sentence: bool = False, save_path: Union[str, os.PathLike, None] = None,
        text_bert: Optional[np.ndarray] = None, sampler=None) -> np.ndarray:
    """Internal.py:265-310, synchronous; returns audio f32 [1280*G] at 32 kHz."""
    if play or split_sentence:
        raise NotImplementedError("playback and sentence splitting are outside the engine (TTSPlayer)")
    if character_name not in _reference_audios:
        raise ValueError("Please call 'set_reference_audio' first to set the reference audio.")
    m = model_manager.get(character_name)
    if m is None:
        raise ValueError(f"character '{character_name}' is not loaded")
    audio = tts_client.tts(text if isinstance(text, str) else np.asarray(text, np.int64),
                           _reference_audios[character_name], m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER,
                           m.T2S_STAGE_DECODER, m.VITS, m.PROMPT_ENCODER, m.LANGUAGE, text_bert=text_bert,
                           g2p=_g2p, sampler=sampler)
    if save_path:
        _write_wav(os.fspath(save_path), audio)
    return audio


def stop() -> None:
    tts_client.stop_event.set()
