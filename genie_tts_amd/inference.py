"""GENIE inference driver (hot path), mirroring src/genie_tts/Core/Inference.py.

`GENIE.tts` has the reference's signature (Inference.py:16-61): it takes the
reference-audio features and the five sessions of a `GSVModel`, runs T2S, the
EOS filter and the vocoder, and returns `audio f32 [1280*G]`.  When the
sessions are this package's engine-backed ones (always, through
`model_manager`), T2S is one `gsv_t2s_generate` call: encoder, prefill, the
whole decode loop as one persistent kernel launch (per-step hipGraphs only as
the fp16-range / co-residency fallback), and the reference's trim + EOS filter
(Inference.py:41-44,108-109) -- no per-step host round trip.
`GENIE.t2s_cpu` is the reference's own session-by-session loop
(Inference.py:63-109) over the same sessions, kept for parity tests.

G2P (`get_phones_and_bert`, src/genie_tts/GetPhonesAndBert.py) is outside this
path: `tts` accepts phoneme ids (+ BERT features) directly, or text together
with a caller-supplied `g2p(text, language) -> (text_seq [1,S] i64, text_bert
[S,1024] f32)` -- e.g. the reference's own function.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Union

import numpy as np

from .engine import EngineStopped, Sampler, request_stop_all
from .sessions import (EncoderSession, FirstStageDecoderSession, StageDecoderSession, VitsSession,
                       PromptEncoderSession)

EOS = 1024
MAX_STEPS = 500          # Inference.py:95


@dataclass
class ReferenceAudio:
    """Reference-audio features (the fields GENIE.tts reads from the reference's
    ReferenceAudio, src/genie_tts/Audio/ReferenceAudio.py:28-76).  api.set_reference_audio
    fills them from a clip: audio.py reads and resamples it (a polyphase restatement of
    soxr HQ), CN-HuBERT (gsv_hubert) gives ssl_content and, for V2ProPlus, the SV model
    (gsv_sv) gives sv_emb -- both on the engine; or the caller supplies them."""
    phonemes_seq: np.ndarray             # i64 [1, R]
    text_bert: np.ndarray                # f32 [R, 1024]
    audio_32k: np.ndarray                # f32 [1, N32]
    ssl_content: np.ndarray              # f32 [1, 768, H]
    sv_emb: Optional[np.ndarray] = None  # f32 [1, 20480] (V2ProPlus)
    global_emb: Optional[np.ndarray] = None
    global_emb_advanced: Optional[np.ndarray] = None
    text: str = ""
    audio_16k: Optional[np.ndarray] = None               # f32 [1, N16] (set_reference_audio)
    sv_fn: Optional[Callable] = None                     # speaker-verification model, audio_16k -> sv_emb

    def update_global_emb(self, prompt_encoder) -> None:
        """ReferenceAudio.py:68-76 (cached after the first call)."""
        if self.global_emb is not None:
            return
        if self.sv_emb is None and self.sv_fn is not None and self.audio_16k is not None:
            self.sv_emb = np.asarray(self.sv_fn(self.audio_16k), np.float32).reshape(1, -1)
        if self.sv_emb is None:
            raise ValueError("V2ProPlus needs the speaker-verification embedding (sv_emb) of the reference: "
                             "load_sv_model(), set_sv_extractor() or pass sv_emb")
        self.global_emb, self.global_emb_advanced = prompt_encoder.run(None, {
            "ref_audio": self.audio_32k, "sv_emb": self.sv_emb})


def eos_filter(semantic_tokens: np.ndarray) -> np.ndarray:
    """Inference.py:41-44: cut at the first id >= 1024."""
    idx = np.where(semantic_tokens >= EOS)
    if len(idx[0]) > 0:
        semantic_tokens = semantic_tokens[..., :idx[-1][0]]
    return semantic_tokens


def _engine_of(*sessions):
    engines = {id(getattr(s, "engine", None)) for s in sessions}
    if len(engines) == 1 and all(isinstance(s, (EncoderSession, FirstStageDecoderSession, StageDecoderSession,
                                                VitsSession)) for s in sessions):
        return sessions[0].engine
    return None


class StopEvent(threading.Event):
    """GENIE.stop_event (Inference.py:13-14): a threading.Event whose set()/clear() also
    set/clear the stop word of every engine (gsv_request_stop), so a decode running on
    the device leaves within two loop steps, as the reference's per-step check
    (Inference.py:96-97) does."""

    def set(self):
        super().set()
        request_stop_all(True)

    def clear(self):
        super().clear()
        request_stop_all(False)


class GENIE:
    def __init__(self):
        self.stop_event = StopEvent()

    def tts(self, text: Union[str, np.ndarray], prompt_audio: ReferenceAudio, encoder, first_stage_decoder,
            stage_decoder, vocoder, prompt_encoder=None, language: str = "japanese",
            text_bert: Optional[np.ndarray] = None, g2p: Optional[Callable] = None,
            sampler: Optional[Sampler] = None) -> Optional[np.ndarray]:
        if isinstance(text, str):
            if g2p is None:
                raise ValueError("text input needs a g2p(text, language) callable (G2P is outside this engine)")
            text_seq, text_bert = g2p("。" + text, language)          # Inference.py:27-28
        else:
            text_seq = np.asarray(text, np.int64).reshape(1, -1)
            if text_bert is None:
                text_bert = np.zeros((text_seq.shape[1], 1024), np.float32)
        eng = _engine_of(encoder, first_stage_decoder, stage_decoder, vocoder)
        if eng is not None:
            sem = self.t2s(prompt_audio.phonemes_seq, prompt_audio.text_bert, text_seq, text_bert,
                           prompt_audio.ssl_content, eng, sampler or first_stage_decoder.sampler)
            if sem is None:            # stopped (Inference.py:96-97)
                return None
        else:
            sem = self.t2s_cpu(prompt_audio.phonemes_seq, prompt_audio.text_bert, text_seq, text_bert,
                               prompt_audio.ssl_content, encoder, first_stage_decoder, stage_decoder)
            if sem is None:
                return None
            sem = eos_filter(sem)
        if prompt_encoder is None:
            return vocoder.run(None, {"text_seq": text_seq, "pred_semantic": sem,
                                      "ref_audio": prompt_audio.audio_32k})[0]
        prompt_audio.update_global_emb(prompt_encoder)
        return vocoder.run(None, {"text_seq": text_seq, "pred_semantic": sem, "ge": prompt_audio.global_emb,
                                  "ge_advanced": prompt_audio.global_emb_advanced})[0]

    def tts_stream(self, texts: Sequence[Union[str, np.ndarray]], prompt_audio: ReferenceAudio, encoder,
                   first_stage_decoder, stage_decoder, vocoder, prompt_encoder=None, language: str = "japanese",
                   text_bert: Optional[np.ndarray] = None, g2p: Optional[Callable] = None,
                   sampler: Optional[Sampler] = None, vocoder_cus: int = 64):
        """tts over a list of sentences, yielding each sentence's audio in order (the
        reference runs them one after the other: TTSPlayer._tts_worker_loop,
        Core/TTSPlayer.py:56-107).  Engine-backed sessions pipeline them: sentence i's
        vocoder runs on `vocoder_cus` CUs of its own while sentence i+1's T2S runs on
        the rest (gsv_vits_decode_async), and sentence i+1's encoder + prefill run on
        those CUs during sentence i's decode (gsv_t2s_prefetch), so sentence i is
        yielded once sentence i+1's T2S is done.  Same tokens and audio as calling
        tts per sentence."""
        eng = _engine_of(encoder, first_stage_decoder, stage_decoder, vocoder)
        if eng is None or vocoder_cus <= 0 or len(texts) < 2:
            for t in texts:
                if self.stop_event.is_set():
                    return
                yield self.tts(t, prompt_audio, encoder, first_stage_decoder, stage_decoder, vocoder, prompt_encoder,
                               language, text_bert, g2p, sampler)
            return
        prev_cus = eng.vocoder_cus     # restored when the stream ends: later single-sentence and
        if prev_cus != vocoder_cus:    # batched calls keep every CU (decode groups, lanes)
            eng.set_vocoder_cus(vocoder_cus)
        try:
            if prompt_encoder is None:
                cond = (vocoder.v2_cond(prompt_audio.audio_32k) if getattr(vocoder, "engine", None) is eng
                        else {"ref_audio": prompt_audio.audio_32k})
            else:
                prompt_audio.update_global_emb(prompt_encoder)
                cond = {"ge": prompt_audio.global_emb, "ge_advanced": prompt_audio.global_emb_advanced}
        except BaseException:          # e.g. a V2ProPlus clip without sv_emb: the CU split is undone
            if eng.vocoder_cus != prev_cus:
                eng.set_vocoder_cus(prev_cus)
            raise
        # every sentence's inputs up front: sentence i+1's T2S is queued behind sentence
        # i's, its encoder + prefill run on the vocoder CUs while sentence i decodes
        seqs = []
        for t in texts:
            if isinstance(t, str):
                if g2p is None:
                    raise ValueError("text input needs a g2p(text, language) callable (G2P is outside this engine)")
                seqs.append(g2p("。" + t, language))
            else:
                ts = np.asarray(t, np.int64).reshape(1, -1)
                seqs.append((ts, text_bert if text_bert is not None else np.zeros((ts.shape[1], 1024), np.float32)))
        ssl = np.asarray(prompt_audio.ssl_content, np.float32).reshape(768, -1)
        utts = [(prompt_audio.phonemes_seq, ts, prompt_audio.text_bert, tb, ssl) for ts, tb in seqs]
        sp = sampler or first_stage_decoder.sampler
        pending = None
        n = len(utts)
        try:
            eng.t2s_prefetch(utts[1], sp)          # launched beside sentence 0's decode
            eng.t2s_generate_start(utts[0], sp)
            for i, (text_seq, _) in enumerate(seqs):
                if self.stop_event.is_set():
                    break
                if i + 1 < n:                      # queued behind sentence i's decode
                    if i + 2 < n:
                        eng.t2s_prefetch(utts[i + 2], sp)
                    eng.t2s_generate_start(utts[i + 1], sp)
                try:
                    sem = eng.t2s_generate_finish().reshape(1, 1, -1)
                except EngineStopped:          # stop_event during sentence i's decode
                    break
                if pending is not None:
                    eng.vits_wait()
                    done, pending = pending, None
                    yield done.cpu().numpy()
                G = sem.size
                eps = vocoder.eps_fn(G) if vocoder.eps_fn else None
                item = dict(text_seq=text_seq, pred_semantic=sem, **cond)
                if eps is not None:
                    item["eps"] = eps
                else:
                    seed = vocoder.next_seed()
                    if seed is not None:
                        item["noise_seed"] = seed
                pending = eng.vits_decode_async(item, vocoder.noise_scale)
            if pending is not None:
                eng.vits_wait()
                done, pending = pending, None
                yield done.cpu().numpy()
        finally:   # stopped, failed or abandoned: started generates and the vocoder call complete
            while getattr(eng, "_gq", None):
                try:
                    eng.t2s_generate_finish()
                except Exception:
                    break
            if pending is not None:
                eng.vits_wait()
            if eng.vocoder_cus != prev_cus:
                eng.set_vocoder_cus(prev_cus)

    def t2s(self, ref_seq, ref_bert, text_seq, text_bert, ssl_content, engine,
            sampler: Sampler) -> Optional[np.ndarray]:
        """Whole T2S on the device; returns the trimmed, EOS-filtered [1,1,G] tokens, or
        None when stop_event interrupted it (Inference.py:96-97)."""
        try:
            tok = engine.t2s_generate([(ref_seq, text_seq, ref_bert, text_bert,
                                        np.asarray(ssl_content, np.float32).reshape(768, -1))], sampler)[0]
        except EngineStopped:
            return None
        return tok.reshape(1, 1, -1)

    def t2s_cpu(self, ref_seq, ref_bert, text_seq, text_bert, ssl_content, encoder, first_stage_decoder,
                stage_decoder) -> Optional[np.ndarray]:
        """The reference's loop (Inference.py:63-109) over session objects."""
        x, prompts = encoder.run(None, {"ref_seq": ref_seq, "text_seq": text_seq, "ref_bert": ref_bert,
                                        "text_bert": text_bert, "ssl_content": ssl_content})
        y, y_emb, *present = first_stage_decoder.run(None, {"x": x, "prompts": prompts})
        names: List[str] = [i.name for i in stage_decoder.get_inputs()]
        idx = 0
        for idx in range(0, MAX_STEPS):
            if self.stop_event.is_set():
                return None
            outs = stage_decoder.run(None, dict(zip(names, [y, y_emb, *present])))
            y, y_emb, stop, *present = outs
            if stop:
                break
        y[0, -1] = 0
        return np.expand_dims(y[:, -idx:], axis=0)

    def tts_batch(self, items: Sequence[tuple], prompt_audio: ReferenceAudio, model, sampler: Sampler) -> List[np.ndarray]:
        """Batched synthesis for one character and reference: items are
        (text_seq, text_bert|None[, force_steps]).  All sequences decode together
        (one multi-sequence persistent launch, ragged: a finished sequence drops out);
        the vocoder runs each utterance's text/flow part on concurrent lanes and the
        generator once over the whole batch (gsv_vits_decode_batch)."""
        toks = self.tts_batch_t2s(items, prompt_audio, model, sampler)
        wavs = self.tts_batch_vocoder(items, toks, prompt_audio, model)
        return [w if isinstance(w, np.ndarray) else w.cpu().numpy() for w in wavs]

    def tts_batch_t2s(self, items: Sequence[tuple], prompt_audio: ReferenceAudio, model, sampler: Sampler):
        """The T2S half of tts_batch: one ragged batched generate -> token arrays."""
        ssl = np.asarray(prompt_audio.ssl_content, np.float32).reshape(768, -1)
        utts = [(prompt_audio.phonemes_seq, it[0], prompt_audio.text_bert, it[1], ssl,
                 it[2] if len(it) > 2 else 0) for it in items]
        # one generate for the whole batch: the engine's multi-sequence persistent decode
        # (B <= 64) costs ~2 ms per extra sequence over a single one
        # (profiles/r03i_batch_sweep.json), so splitting never pays
        return model.ENGINE.t2s_generate(utts, sampler)

    def tts_batch_vocoder(self, items: Sequence[tuple], toks, prompt_audio: ReferenceAudio, model,
                          overlapped: bool = False):
        """The vocoder half of tts_batch.  overlapped=True (engine-backed vocoder only) starts
        the batch on the vocoder lanes and returns device tensors that are valid after
        model.ENGINE.vits_batch_wait(); the T2S of the next batch runs beside it
        (gsv_vits_decode_batch_async)."""
        eng = model.ENGINE
        if model.PROMPT_ENCODER is not None:
            prompt_audio.update_global_emb(model.PROMPT_ENCODER)
        cond = ({"ref_audio": prompt_audio.audio_32k} if model.PROMPT_ENCODER is None else
                {"ge": prompt_audio.global_emb, "ge_advanced": prompt_audio.global_emb_advanced})
        if model.PROMPT_ENCODER is None and getattr(model.VITS, "engine", None) is eng:
            cond = model.VITS.v2_cond(prompt_audio.audio_32k)   # the reference branch once per reference
        if getattr(model.VITS, "engine", None) is not eng:
            return [model.VITS.run(None, {"text_seq": it[0], "pred_semantic": tok.reshape(1, 1, -1), **cond})[0]
                    for it, tok in zip(items, toks)]
        # engine-backed vocoder: all utterances on concurrent lanes (gsv_vits_decode_batch)
        batch = [dict(text_seq=it[0], pred_semantic=tok, noise_seed=model.VITS.next_seed(), **cond)
                 for it, tok in zip(items, toks)]
        if overlapped:
            return eng.vits_decode_batch_async(batch, model.VITS.noise_scale)
        return eng.vits_decode_batch(batch, model.VITS.noise_scale)


tts_client = GENIE()
