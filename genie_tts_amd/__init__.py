"""MI355X-native GPT-SoVITS inference engine (the Genie-TTS synthesis hot path).

The product is libgenie_engine.so (C ABI, include/genie_engine.h) built from
genie_tts_amd/csrc; this package is its host side: ctypes bindings (engine),
onnxruntime-session-shaped objects (sessions), the character cache
(model_manager), the reference's inference driver (inference) and the
`genie_tts` entry points (api).  There is no CPU fallback.
"""
from .api import (clear_reference_audio_cache, load_character, load_cn_hubert, load_roberta, load_sv_model,  # noqa: F401
                  load_weights, set_g2p,
                  set_reference_audio, set_reference_features, set_ssl_extractor, set_sv_extractor, stop, tts,
                  tts_async, unload_character, wait_for_playback_done)

__all__ = ["load_character", "load_cn_hubert", "load_roberta", "load_sv_model", "load_weights", "unload_character", "set_reference_audio", "set_reference_features",
           "set_g2p", "set_ssl_extractor", "set_sv_extractor", "tts", "tts_async", "stop", "wait_for_playback_done",
           "clear_reference_audio_cache"]
