"""CPU: host-side semantics and the C ABI library (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trim_semantics():
    """Inference.py:108-109 then :41-44."""
    from oracle.restate import trim_tokens
    y = [5, 6, 7, 100, 200, 300]                 # P=3 prompts, g0=100, loop tokens 200, 300
    # stop fired at idx=1 (2nd loop step): keep y[-1:] after zeroing the last
    np.testing.assert_array_equal(trim_tokens(y, 1), np.array([[[0]]]))
    np.testing.assert_array_equal(trim_tokens(y, 2), np.array([[[200, 0]]]))
    # idx == 0: y[:, -0:] is the whole y
    np.testing.assert_array_equal(trim_tokens(y, 0), np.array([[[5, 6, 7, 100, 200, 0]]]))
    # an EOS inside the kept window truncates at its first occurrence
    np.testing.assert_array_equal(trim_tokens([1, 2, 1024, 9, 9], 3), np.array([[[1024, 9, 0]]])[..., :0])
    np.testing.assert_array_equal(trim_tokens([1, 2, 3, 1024, 9], 3), np.array([[[3]]]))


def test_engine_trim_matches_oracle():
    """The C++ trim (gsv_t2s_generate) restates the same rule; check it on the host copy."""
    from oracle.restate import trim_tokens
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = int(rng.integers(3, 40))
        y = rng.integers(0, 1025, size=n).tolist()
        idx = int(rng.integers(0, n - 1))
        ref = trim_tokens(y, idx).reshape(-1).tolist()
        yy = list(y)
        yy[-1] = 0
        start = n - idx if idx > 0 else 0
        cnt = n - start
        for i in range(cnt):
            if yy[start + i] >= 1024:
                cnt = i
                break
        assert yy[start:start + cnt] == ref


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "genie_engine.h")).read()
    return sorted(set(re.findall(r"\b(gsv_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    from genie_tts_amd.build import LIB, build
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    missing = [f for f in _header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    from genie_tts_amd import engine
    assert set(engine.EXPORTED) <= set(_header_functions())
    assert lib.gsv_version


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from genie_tts_amd.engine import Engine, EngineError
    with pytest.raises(EngineError, match="no CPU fallback"):
        Engine({}, "v2")


def test_eos_filter_semantics():
    """inference.eos_filter restates Inference.py:41-44."""
    from genie_tts_amd.inference import eos_filter
    a = np.array([[[3, 5, 1024, 7, 1024]]])
    np.testing.assert_array_equal(eos_filter(a), np.array([[[3, 5]]]))
    b = np.array([[[3, 5, 7]]])
    np.testing.assert_array_equal(eos_filter(b), b)
    np.testing.assert_array_equal(eos_filter(np.array([[[1024, 1]]])).shape, (1, 1, 0))


def test_session_interfaces_match_templates():
    """Input/output names and order of the session shims = SURVEY Appendix A."""
    from genie_tts_amd import sessions as S
    st = [i.name for i in S.StageDecoderSession.INPUTS]
    assert st[:2] == ["iy", "iy_emb"] and len(st) == 50
    assert st[2:6] == ["past_k_layer_0", "past_v_layer_0", "past_k_layer_1", "past_v_layer_1"]
    so = [o.name for o in S.StageDecoderSession.OUTPUTS]
    assert so[:3] == ["y", "y_emb", "stop_condition_tensor"] and so[3] == "present_k_layer_0"
    assert [i.name for i in S.EncoderSession.INPUTS] == ["ref_seq", "text_seq", "ref_bert", "text_bert",
                                                         "ssl_content"]
    assert [o.name for o in S.FirstStageDecoderSession.OUTPUTS][:2] == ["y", "y_emb"]
    assert [i.name for i in S.PromptEncoderSession.INPUTS] == ["ref_audio", "sv_emb"]


def test_api_requires_reference_and_gpu():
    import genie_tts_amd as G
    assert G.tts("nobody", [3, 4, 5]) is None            # Internal.py:292-294: logs, returns
    with pytest.raises(ValueError):
        G.load_character("x", "/nonexistent", "klingon")


def test_fp16_only_weight_paths_refuse_fp32_values():
    """The engine's fp16-only loaders (up_f16 / up_f16_t) refuse any value that is not
    fp16-exact instead of rounding it; gsv_f16_exact is the check they apply."""
    from genie_tts_amd.build import LIB, build
    if not os.path.exists(LIB):
        build()
    from genie_tts_amd import engine
    h = np.array([0.5, -3.25, 65504.0, 2.0 ** -24, 0.0], np.float32)
    assert engine.f16_exact(h) == -1
    w = h.copy()
    w[3] = np.float32(0.1)                       # 0.1 has no fp16 representation
    assert engine.f16_exact(w) == 3
    assert engine.f16_exact(np.float32([1.0 + 2.0 ** -20])) == 0
    assert engine.f16_exact(np.zeros(0, np.float32)) == -1
    # the synthetic RoBERTa of the tests carries fp32 values, as RoBERTa.onnx does
    from genie_tts_amd import synth, weights as W
    q = synth.synth_tensor("encoder.layer.0.attention.self.query.weight", (1024, 1024), fp16=False)
    assert engine.f16_exact(q) >= 0


def test_hbm_copy_probe_rejects_bad_arguments_without_touching_the_gpu():
    """gsv_debug_hbm_copy (bench.py's achievable-HBM probe) checks its arguments before any HIP call."""
    from genie_tts_amd import engine
    L = engine.lib()
    ms = ctypes.c_float(0.0)
    assert L.gsv_debug_hbm_copy(None, None, 1 << 20, 10, None, ctypes.byref(ms)) != 0
    assert L.gsv_debug_hbm_copy(ctypes.c_void_p(16), ctypes.c_void_p(32), 100, 10, None, ctypes.byref(ms)) != 0
    assert b"16-B aligned" in L.gsv_last_error()
