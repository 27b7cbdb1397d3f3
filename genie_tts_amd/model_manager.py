"""Per-character engine + session cache, mirroring the reference's ModelManager.

Reference: src/genie_tts/ModelManager.py:39-56 (GSVModel), :116-319 (ModelManager:
LRU of characters, `Max_Cached_Character_Models` env, load_character/get/
has_character/remove_character/remove_all_character).  Instead of five
onnxruntime sessions per character, one `Engine` per character holds the
device weights (read from the same converted character directory: ONNX
initializer table + fp16/fp32 bins, ModelManager.py:59-114) and the five
session objects of `sessions.py` share it.
"""
from __future__ import annotations

import gc
import logging
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Optional, Union

import numpy as np

from . import weights as W
from .engine import Engine, Sampler, make_sampler
from .sessions import (EncoderSession, FirstStageDecoderSession, PromptEncoderSession,
                       StageDecoderSession, VitsSession, _T2SState)

logger = logging.getLogger(__name__)


@dataclass
class GSVModel:
    """Same fields as the reference's GSVModel (ModelManager.py:48-56)."""
    LANGUAGE: str
    T2S_ENCODER: EncoderSession
    T2S_FIRST_STAGE_DECODER: FirstStageDecoderSession
    T2S_STAGE_DECODER: StageDecoderSession
    VITS: VitsSession
    PROMPT_ENCODER: Optional[PromptEncoderSession] = None
    PROMPT_ENCODER_PATH: Optional[str] = None
    ENGINE: Optional[Engine] = None
    VERSION: str = "v2"


def build_model(weights: Dict[str, Dict[str, np.ndarray]], version: str, language: str = "Japanese",
                device: int = 0, sampler: Optional[Sampler] = None, model_dir: Optional[str] = None,
                pe_div_term: Optional[np.ndarray] = None, vits_noise: str = "philox") -> GSVModel:
    eng = Engine(weights, version, device=device, pe_div_term=pe_div_term)
    emb = np.asarray(weights["t2s"]["ar_audio_embedding.word_embeddings.weight"], np.float32)
    st = _T2SState()
    sp = sampler or make_sampler(greedy=False)
    pe = PromptEncoderSession(eng) if "prompt_encoder" in weights else None
    return GSVModel(
        LANGUAGE=language,
        T2S_ENCODER=EncoderSession(eng),
        T2S_FIRST_STAGE_DECODER=FirstStageDecoderSession(eng, emb, st, sp),
        T2S_STAGE_DECODER=StageDecoderSession(eng, emb, st, sp),
        VITS=VitsSession(eng, version, noise=vits_noise),
        PROMPT_ENCODER=pe,
        PROMPT_ENCODER_PATH=os.path.join(model_dir, "prompt_encoder_fp32.onnx") if (model_dir and pe) else None,
        ENGINE=eng,
        VERSION=version,
    )


class ModelManager:
    def __init__(self, device: int = 0):
        self.capacity = int(os.getenv("Max_Cached_Character_Models", "3"))
        self.device = device
        self.character_to_model: "OrderedDict[str, GSVModel]" = OrderedDict()
        self.character_to_language: Dict[str, str] = {}
        self.character_model_paths: Dict[str, str] = {}
        self.sampler: Optional[Sampler] = None
        self.vits_noise = "philox"       # z_p noise of new characters' vocoders ("zero": deterministic tests)
        self.cn_hubert = None            # HubertSession (ModelManager.py:127,172-195)
        self.roberta = None              # RobertaSession (ModelManager.py:129,132-150)
        self.speaker_verification_model = None   # SvSession (ModelManager.py:128,155-170)

    def _put(self, name: str, model: GSVModel) -> None:
        self.character_to_model[name] = model
        self.character_to_model.move_to_end(name)
        while len(self.character_to_model) > self.capacity:
            _, old = self.character_to_model.popitem(last=False)
            if old.ENGINE is not None:
                old.ENGINE.close()

    def load_character(self, character_name: str, model_dir: str, language: str) -> bool:
        """Reads the converted character directory (same files as the reference)."""
        name = character_name.lower()
        if name in self.character_to_model:
            self.character_to_model.move_to_end(name)
            return True
        version, w = W.load_character_weights(model_dir)
        self._put(name, build_model(w, version, language, self.device, self.sampler, model_dir,
                                    vits_noise=self.vits_noise))
        self.character_to_language[name] = language
        self.character_model_paths[name] = model_dir
        logger.info("Character %s loaded (%s) from %s", name, "V2ProPlus" if version != "v2" else "V2", model_dir)
        return True

    def load_weights(self, character_name: str, weights: Dict[str, Dict[str, np.ndarray]], version: str,
                     language: str = "Japanese") -> bool:
        """Register a character from in-memory weights (synthetic characters, tests, benchmarks)."""
        name = character_name.lower()
        self._put(name, build_model(weights, version, language, self.device, self.sampler,
                                    vits_noise=self.vits_noise))
        self.character_to_language[name] = language
        return True

    def load_cn_hubert(self, model: Union[str, Dict[str, np.ndarray], None] = None) -> bool:
        """CN-HuBERT on its own engine (`g/ModelManager.py:172-195`): `model` is the
        GenieData/chinese-hubert-base directory or in-memory weights (hubert_spec
        names); default: $HUBERT_MODEL_DIR."""
        if self.cn_hubert is not None:
            return True
        from .sessions import HubertSession
        if model is None:
            model = os.getenv("HUBERT_MODEL_DIR")
            if not model:
                raise FileNotFoundError("CN-HuBERT: pass a directory or weights, or set HUBERT_MODEL_DIR")
        w = W.load_hubert_weights(model) if isinstance(model, (str, os.PathLike)) else model
        self.cn_hubert = HubertSession(Engine({"hubert": w}, "v2", device=self.device))
        logger.info("CN-HuBERT loaded")
        return True

    def load_roberta_model(self, model: Union[str, Dict[str, np.ndarray], None] = None) -> bool:
        """RoBERTa on its own engine (`g/ModelManager.py:132-150`): `model` is the
        GenieData RoBERTa directory or in-memory weights (roberta_spec names);
        default: $ROBERTA_MODEL_DIR."""
        if self.roberta is not None:
            return True
        from .sessions import RobertaSession
        if model is None:
            model = os.getenv("ROBERTA_MODEL_DIR")
            if not model:
                raise FileNotFoundError("RoBERTa: pass a directory or weights, or set ROBERTA_MODEL_DIR")
        w = W.load_roberta_weights(model) if isinstance(model, (str, os.PathLike)) else model
        self.roberta = RobertaSession(Engine({"roberta": w}, "v2", device=self.device))
        logger.info("RoBERTa loaded")
        return True

    def load_sv_model(self, model: Union[str, Dict[str, np.ndarray], None] = None) -> bool:
        """Speaker verification on its own engine (`g/ModelManager.py:155-170`): `model`
        is GenieData's speaker_encoder.onnx (or its directory) or in-memory weights
        (sv_spec names); default: $SV_MODEL_PATH."""
        if self.speaker_verification_model is not None:
            return True
        from .sessions import SvSession
        if model is None:
            model = os.getenv("SV_MODEL_PATH")
            if not model:
                raise FileNotFoundError("SV model: pass speaker_encoder.onnx or weights, or set SV_MODEL_PATH")
        w = W.load_sv_weights(model) if isinstance(model, (str, os.PathLike)) else model
        self.speaker_verification_model = SvSession(Engine({"sv": w}, "v2", device=self.device))
        logger.info("Speaker Verification model loaded")
        return True

    def unload_sv_model(self) -> None:
        if self.speaker_verification_model is not None:
            self.speaker_verification_model.engine.close()
            self.speaker_verification_model = None

    def unload_cn_hubert(self) -> None:
        if self.cn_hubert is not None:
            self.cn_hubert.engine.close()
            self.cn_hubert = None

    def get(self, character_name: str) -> Optional[GSVModel]:
        name = character_name.lower()
        if name in self.character_to_model:
            self.character_to_model.move_to_end(name)
            return self.character_to_model[name]
        if name in self.character_model_paths:          # evicted: reload from disk
            if self.load_character(name, self.character_model_paths[name],
                                   self.character_to_language.get(name, "Japanese")):
                return self.character_to_model[name]
            del self.character_model_paths[name]
        return None

    def has_character(self, character_name: str) -> bool:
        name = character_name.lower()
        return name in self.character_model_paths or name in self.character_to_model

    def remove_character(self, character_name: str) -> None:
        name = character_name.lower()
        m = self.character_to_model.pop(name, None)
        if m is not None and m.ENGINE is not None:
            m.ENGINE.close()
        gc.collect()

    def remove_all_character(self) -> None:
        for n in list(self.character_to_model):
            self.remove_character(n)


model_manager = ModelManager()
