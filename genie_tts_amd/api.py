"""The `genie_tts` entry points this engine serves (src/genie_tts/__init__.py:1-28,
src/genie_tts/Internal.py:94-330), restricted to the synthesis hot path.

Same names, argument meaning and defaults as the reference:
  load_character(character_name, onnx_model_dir, language)        Internal.py:94-126
  set_reference_audio(character_name, audio_path, audio_text, language=None)
                                                                   Internal.py:143-190
  tts(character_name, text, play=False, split_sentence=True, save_path=None)
                                                                   Internal.py:265-310
  tts_async(character_name, text, play=False, split_sentence=False, save_path=None)
      -> async iterator of 16-bit PCM bytes, one chunk per sentence Internal.py:193-262
  unload_character, clear_reference_audio_cache, stop, wait_for_playback_done

What the engine does not contain (outside the hot path) is pluggable:
  set_g2p(fn(text, language) -> (phones i64 [1,S], bert f32 [S,1024]))   -- G2P (+ BERT), or
          -> (phones, None, input_ids, word2ph): RoBERTa then runs on the engine (load_roberta)
  set_ssl_extractor(fn(audio_16k [1,N]) -> ssl_content [1,768,H])       -- CN-HuBERT override
  set_sv_extractor(fn(audio_16k [1,N]) -> sv_emb [1,20480])             -- V2ProPlus SV model
CN-HuBERT itself runs on the engine (gsv_hubert) once load_cn_hubert(dir | weights) has
been called or $HUBERT_MODEL_DIR is set (ModelManager.py:172-195),
or the features can be passed to set_reference_audio directly (phonemes_seq=,
text_bert=, ssl_content=, sv_emb=).  Reading/resampling the clip is audio.py
(own WAV/AIFF reader + polyphase resampler: soundfile/soxr are absent).
Differences: `tts` also returns the audio; `play=True` has no output device in
this environment and is skipped with a warning, as the reference does when
sounddevice fails (Core/TTSPlayer.py:136-146).
"""
from __future__ import annotations

import asyncio
import logging
import os
import threading
from collections import OrderedDict
from typing import AsyncIterator, Callable, Dict, List, Optional, Sequence, Union

import numpy as np

from . import audio as A
from .inference import ReferenceAudio, tts_client
from .model_manager import model_manager
from .text_splitter import TextSplitter

logger = logging.getLogger(__name__)

SAMPLE_RATE = 32000
# CUs reserved for the overlapped vocoder of multi-sentence synthesis (0: sequential)
VOCODER_CUS = int(os.environ.get("GENIE_VOCODER_CUS", "64"))
SUPPORTED_AUDIO_EXTS = A.SUPPORTED_AUDIO_EXTS
_reference_audios: Dict[str, ReferenceAudio] = {}
_clip_cache: "OrderedDict[str, ReferenceAudio]" = OrderedDict()   # ReferenceAudio._prompt_cache (LRU 10)
_g2p: Optional[Callable] = None
_ssl_extractor: Optional[Callable] = None
_sv_extractor: Optional[Callable] = None
# The player's session stop (TTSPlayer._stop_event, Core/TTSPlayer.py:208-222): set by stop(),
# cleared when a tts / tts_async session starts (TTSPlayer.start_session, :175).  A stopped
# session synthesizes no further sentence and saves nothing; tts_client.stop_event (GENIE's)
# is the per-sentence word that abandons a running decode, cleared per sentence as the
# worker loop does (:86).
_session_stop = threading.Event()


def _norm_language(language: Optional[str]) -> str:
    if language is None:
        return "Japanese"
    l = language.lower()
    return {"ja": "Japanese", "jp": "Japanese", "japanese": "Japanese", "en": "English", "english": "English",
            "zh": "Chinese", "chinese": "Chinese", "hybrid": "Hybrid-Chinese-English",
            "hybrid-chinese-english": "Hybrid-Chinese-English"}.get(l, language)


def set_g2p(fn: Optional[Callable]) -> None:
    """fn(text, language) -> (text_seq i64 [1,S], text_bert f32 [S,1024])."""
    global _g2p
    _g2p = fn


def set_ssl_extractor(fn: Optional[Callable]) -> None:
    """fn(audio_16k f32 [1,N]) -> ssl_content f32 [1,768,H] (the reference's CN-HuBERT session)."""
    global _ssl_extractor
    _ssl_extractor = fn


def load_cn_hubert(model=None) -> None:
    """CN-HuBERT weights: the GenieData/chinese-hubert-base directory or a dict of
    arrays (weights.hubert_spec names); `g/ModelManager.py:172-195`."""
    model_manager.load_cn_hubert(model)


def load_roberta(model=None) -> None:
    """RoBERTa (chinese-roberta-wwm-ext-large) weights: the GenieData RoBERTa directory
    or a dict of arrays (weights.roberta_spec names); `g/ModelManager.py:132-150`."""
    model_manager.load_roberta_model(model)


def load_sv_model(model=None) -> None:
    """Speaker-verification weights (V2ProPlus sv_emb): GenieData speaker_encoder.onnx
    (or its directory) or a dict of arrays (weights.sv_spec names); runs on the engine
    (gsv_sv).  `g/ModelManager.py:155-170`."""
    model_manager.load_sv_model(model)


def set_sv_extractor(fn: Optional[Callable]) -> None:
    """fn(audio_16k f32 [1,N]) -> sv_emb f32 [1,20480] (the reference's speaker-verification session)."""
    global _sv_extractor
    _sv_extractor = fn


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


def _text_features(text: str, language: str, phonemes_seq=None, text_bert=None):
    if phonemes_seq is None:
        if _g2p is None:
            raise ValueError("no G2P: pass phonemes_seq (and text_bert) or call set_g2p()")
        g = _g2p(text, language)
        phonemes_seq, text_bert = g[0], g[1]
        if len(g) == 4 and text_bert is None and model_manager.roberta is not None:
            # (phones, None, input_ids, word2ph): Chinese BERT features on the engine
            # (GetPhonesAndBert.py:64-74; tokenizing text_clean stays with the G2P)
            ids = np.asarray(g[2], np.int64).reshape(1, -1)
            text_bert = model_manager.roberta.run(None, {"input_ids": ids, "attention_mask": np.ones_like(ids),
                                                         "repeats": np.asarray(g[3], np.int64)})[0]
    ps = np.asarray(phonemes_seq, np.int64).reshape(1, -1)
    tb = np.zeros((ps.shape[1], 1024), np.float32) if text_bert is None else np.asarray(text_bert, np.float32)
    return ps, tb


def set_reference_audio(character_name: str, audio_path: Union[str, os.PathLike], audio_text: str,
                        language: Optional[str] = None, *, phonemes_seq=None, text_bert=None,
                        ssl_content=None, sv_emb=None) -> None:
    """Internal.py:143-190 + ReferenceAudio.py:28-57: the clip at 32 kHz (+0.3 s
    silence) and 16 kHz, the prompt text's phones/BERT, the SSL content of the 16 kHz
    clip; cached per clip path (LRU, Max_Cached_Reference_Audio)."""
    path = os.fspath(audio_path)
    ext = os.path.splitext(path)[1].lower()
    if ext not in SUPPORTED_AUDIO_EXTS:
        logger.error("Audio format '%s' is not supported. Only the following formats are supported: %s", ext,
                     sorted(SUPPORTED_AUDIO_EXTS))
        return
    if language is None:
        m = model_manager.get(character_name)
        if m is None:
            raise ValueError("No language specified")
        language = m.LANGUAGE
    language = _norm_language(language)
    if language not in ("Japanese", "English", "Chinese"):
        raise ValueError("Unknown language")
    ref = _clip_cache.get(path)
    if ref is None:
        audio_32k = A.load_audio(path, 32000).reshape(1, -1)
        audio_16k = A.resample(audio_32k[0], 32000, 16000).reshape(1, -1)
        if ssl_content is None:
            if _ssl_extractor is not None:
                ssl_content = _ssl_extractor(audio_16k)
            elif model_manager.cn_hubert is not None or os.getenv("HUBERT_MODEL_DIR"):
                model_manager.load_cn_hubert()          # ReferenceAudio.py:48-52
                ssl_content = model_manager.cn_hubert.run(None, {"input_values": audio_16k})[0]
            else:
                raise ValueError("no SSL extractor (CN-HuBERT): load_cn_hubert(), pass ssl_content "
                                 "or call set_ssl_extractor()")
        ps, tb = _text_features(audio_text, language, phonemes_seq, text_bert)
        ref = ReferenceAudio(phonemes_seq=ps, text_bert=tb, audio_32k=audio_32k,
                             ssl_content=np.asarray(ssl_content, np.float32).reshape(1, 768, -1),
                             sv_emb=None if sv_emb is None else np.asarray(sv_emb, np.float32).reshape(1, -1),
                             text=audio_text)
        ref.audio_16k = audio_16k
        ref.sv_fn = _sv_extractor
        _clip_cache[path] = ref
        while len(_clip_cache) > int(os.getenv("Max_Cached_Reference_Audio", "10")):
            _clip_cache.popitem(last=False)
    else:
        _clip_cache.move_to_end(path)
        if ref.text != audio_text or phonemes_seq is not None:      # ReferenceAudio.py:18-21 set_text
            ref.phonemes_seq, ref.text_bert = _text_features(audio_text, language, phonemes_seq, text_bert)
            ref.text = audio_text
        if sv_emb is not None:
            ref.sv_emb = np.asarray(sv_emb, np.float32).reshape(1, -1)
            ref.global_emb = ref.global_emb_advanced = None
    _reference_audios[character_name] = ref


def set_reference_features(character_name: str, phonemes_seq: np.ndarray, text_bert: Optional[np.ndarray],
                           audio_32k: np.ndarray, ssl_content: np.ndarray, sv_emb: Optional[np.ndarray] = None,
                           audio_text: str = "") -> None:
    """Set the reference from already-extracted features (the fields GENIE.tts reads)."""
    ps = np.asarray(phonemes_seq, np.int64).reshape(1, -1)
    tb = np.zeros((ps.shape[1], 1024), np.float32) if text_bert is None else np.asarray(text_bert, np.float32)
    _reference_audios[character_name] = ReferenceAudio(
        phonemes_seq=ps, text_bert=tb, audio_32k=np.asarray(audio_32k, np.float32).reshape(1, -1),
        ssl_content=np.asarray(ssl_content, np.float32).reshape(1, 768, -1),
        sv_emb=None if sv_emb is None else np.asarray(sv_emb, np.float32).reshape(1, -1), text=audio_text)


def clear_reference_audio_cache() -> None:
    _reference_audios.clear()
    _clip_cache.clear()


def _sentences(text, split_sentence: bool) -> List:
    if isinstance(text, str):
        return TextSplitter().split(text.strip()) if split_sentence else ([text] if text else [])
    return [np.asarray(text, np.int64)]               # phoneme ids: one utterance


def _ensure_sv_emb(m, ref) -> None:
    """V2ProPlus: the reference clip's speaker embedding, once per clip
    (ReferenceAudio.update_global_emb, `g/Audio/ReferenceAudio.py:68-76`): a plugged
    extractor, else the engine's SV model (load_sv_model() or $SV_MODEL_PATH)."""
    if m.PROMPT_ENCODER is None or ref.sv_emb is not None:
        return
    if getattr(ref, "sv_fn", None) is not None:
        ref.sv_emb = np.asarray(ref.sv_fn(ref.audio_16k), np.float32).reshape(1, -1)
    elif getattr(ref, "audio_16k", None) is not None and (model_manager.speaker_verification_model is not None
                                                          or os.getenv("SV_MODEL_PATH")):
        model_manager.load_sv_model()
        sv = model_manager.speaker_verification_model.run(None, {"waveform": ref.audio_16k})[0]
        ref.sv_emb = np.asarray(sv, np.float32).reshape(1, -1)


def _synthesize(character_name: str, sentence, text_bert=None, sampler=None) -> np.ndarray:
    m = model_manager.get(character_name)
    if m is None:
        raise ValueError(f"character '{character_name}' is not loaded")
    ref = _reference_audios[character_name]
    _ensure_sv_emb(m, ref)
    if _session_stop.is_set():
        return None
    tts_client.stop_event.clear()            # TTSPlayer.py:86, per sentence
    if _session_stop.is_set():               # a stop() between the check and the clear
        tts_client.stop_event.set()
        return None
    return tts_client.tts(sentence, ref, m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER, m.VITS,
                          m.PROMPT_ENCODER, m.LANGUAGE, text_bert=text_bert, g2p=_g2p, sampler=sampler)


def _synthesize_all(character_name: str, sentences: List, text_bert=None, sampler=None):
    """Every sentence, in order; on the engine the vocoder of one sentence overlaps the
    T2S of the next (GENIE.tts_stream)."""
    if len(sentences) < 2:
        return [_synthesize(character_name, s, text_bert, sampler) for s in sentences]
    m = model_manager.get(character_name)
    if m is None:
        raise ValueError(f"character '{character_name}' is not loaded")
    ref = _reference_audios[character_name]
    _ensure_sv_emb(m, ref)
    if _session_stop.is_set():
        return []
    tts_client.stop_event.clear()
    if _session_stop.is_set():
        tts_client.stop_event.set()
        return []
    return list(tts_client.tts_stream(sentences, ref, m.T2S_ENCODER, m.T2S_FIRST_STAGE_DECODER, m.T2S_STAGE_DECODER,
                                      m.VITS, m.PROMPT_ENCODER, m.LANGUAGE, text_bert=text_bert, g2p=_g2p,
                                      sampler=sampler, vocoder_cus=VOCODER_CUS))


def _play(audio: np.ndarray) -> None:
    try:
        import sounddevice as sd   # noqa: F401  (absent here, as on most servers)
        sd.play(np.asarray(audio, np.float32).squeeze(), SAMPLE_RATE)
        sd.wait()
    except Exception as e:      # TTSPlayer.py:136-146: playback skipped, synthesis goes on
        logger.warning("Failed to initialize sounddevice: %s. Audio playback will be skipped.", e)


def tts(character_name: str, text: Union[str, Sequence[int], np.ndarray], play: bool = False,
        split_sentence: bool = True, save_path: Union[str, os.PathLike, None] = None,
        text_bert: Optional[np.ndarray] = None, sampler=None) -> Optional[np.ndarray]:
    """Internal.py:265-310 (TTSPlayer session: split, synthesize each sentence, save the
    concatenation as 16-bit WAV).  Returns the audio f32 [sum 1280*G_i] at 32 kHz."""
    if character_name not in _reference_audios:
        logger.error("Please call 'set_reference_audio' first to set the reference audio.")
        return None
    _session_stop.clear()                    # TTSPlayer.start_session
    chunks = [c for c in _synthesize_all(character_name, _sentences(text, split_sentence), text_bert, sampler)
              if c is not None]
    audio = np.concatenate(chunks) if chunks else np.zeros(0, np.float32)
    if _session_stop.is_set():               # stopped: the session's STREAM_END (and its save) never runs
        return audio
    if save_path:
        A.write_wav(os.fspath(save_path), audio, SAMPLE_RATE)
    if play:
        _play(audio)
    return audio


async def tts_async(character_name: str, text: str, play: bool = False, split_sentence: bool = False,
                    save_path: Union[str, os.PathLike, None] = None) -> AsyncIterator[bytes]:
    """Internal.py:193-262: yields one raw 16-bit PCM chunk per sentence as soon as it
    is synthesized (TTSPlayer chunk callback), the engine running off the event loop."""
    if character_name not in _reference_audios:
        raise ValueError("Please call 'set_reference_audio' first to set the reference audio.")
    loop = asyncio.get_running_loop()
    _session_stop.clear()                    # TTSPlayer.start_session
    chunks = []
    for s in _sentences(text, split_sentence):
        if _session_stop.is_set():
            return
        audio = await loop.run_in_executor(None, _synthesize, character_name, s)
        if _session_stop.is_set():
            # stop() during the sentence: the reference's worker sends chunk_callback(None) and
            # the iterator ends without that chunk (TTSPlayer.py:109-114, Internal.py:258-262)
            return
        if audio is None:
            continue
        chunks.append(audio)
        if play:
            await loop.run_in_executor(None, _play, audio)
        yield A.to_pcm16(audio)
    if save_path and chunks:
        A.write_wav(os.fspath(save_path), np.concatenate(chunks), SAMPLE_RATE)


def wait_for_playback_done() -> None:
    """Playback is synchronous here (see `play`)."""


def stop() -> None:
    """TTSPlayer.stop (Core/TTSPlayer.py:208-222): the running sentence's decode is abandoned
    (GENIE.stop_event -> the engines' stop word) and the session ends: tts returns what was
    synthesized before the stop without saving, a tts_async iterator ends.  The next
    tts / tts_async call starts a new session."""
    _session_stop.set()
    tts_client.stop_event.set()
