"""ctypes binding of libgenie_engine.so (C ABI: include/genie_engine.h).

PyTorch is plumbing here: device buffers are torch tensors whose data_ptr()
is handed to the engine, and calls run on torch's current HIP stream.  There
is no CPU fallback: if the library is missing or fails to load, every entry
point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import weights as W

# GENIE_ENGINE_LIB: an alternative build of the same library (A/B timing of a kernel variant)
_LIB_PATH = os.environ.get("GENIE_ENGINE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                                "libgenie_engine.so")
_lib = None

GSV_F32, GSV_F16 = 0, 1
GSV_V2, GSV_V2PP = 0, 1
MAX_BATCH = 64           # gsv_reserve: sequences decoded together


GSV_E_STOPPED = -6       # a generate abandoned by gsv_request_stop


class EngineError(RuntimeError):
    pass


class EngineStopped(EngineError):
    """A T2S generate was abandoned by a stop request (gsv_request_stop); the reference's
    loop returns None for the sentence then (Inference.py:96-97)."""


# Every live engine, so one stop request reaches them all, and the current request state for
# new engines.  The scope is the process, as in the reference: GENIE.stop_event belongs to the
# module-level tts_client (Core/Inference.py:13-14, 112) that every character shares, so a
# stop() ends the synthesis of every character.  _engines_lock orders registration against
# a stop request arriving from another thread.
_engines: "weakref.WeakSet" = weakref.WeakSet()
_engines_lock = threading.Lock()
_stop_on = False


def request_stop_all(on: bool) -> None:
    """Set (or clear) the stop word of every engine of this process (gsv_request_stop).
    Writes one host word per engine: safe from any thread while a generate runs."""
    global _stop_on
    with _engines_lock:
        _stop_on = bool(on)
        live = list(_engines)
        for e in live:
            if getattr(e, "h", None):
                lib().gsv_request_stop(e.h, int(on))


class Utt(ctypes.Structure):
    _fields_ = [
        ("ref_seq", ctypes.c_void_p), ("n_ref", ctypes.c_int32),
        ("text_seq", ctypes.c_void_p), ("n_text", ctypes.c_int32),
        ("ref_bert", ctypes.c_void_p), ("text_bert", ctypes.c_void_p),
        ("ssl", ctypes.c_void_p), ("n_ssl", ctypes.c_int32),
        ("force_steps", ctypes.c_int32),
    ]


class VitsItem(ctypes.Structure):
    _fields_ = [
        ("text_seq", ctypes.c_void_p), ("n_text", ctypes.c_int32),
        ("sem", ctypes.c_void_p), ("n_sem", ctypes.c_int32),
        ("ref_audio", ctypes.c_void_p), ("n_audio", ctypes.c_int32),
        ("ge", ctypes.c_void_p), ("ge_adv", ctypes.c_void_p),
        ("eps", ctypes.c_void_p), ("noise_seed", ctypes.c_uint64), ("noise_mode", ctypes.c_int32),
        ("audio", ctypes.c_void_p),
    ]


class Sampler(ctypes.Structure):
    _fields_ = [
        ("top_k", ctypes.c_int32), ("temperature", ctypes.c_float),
        ("repetition_penalty", ctypes.c_float), ("greedy", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("max_steps", ctypes.c_int32),
        ("force_steps", ctypes.c_int32),
    ]


def make_sampler(top_k: int = 15, temperature: float = 1.0, repetition_penalty: float = 1.35,
                 greedy: bool = True, seed: int = 1234, max_steps: int = 500,
                 force_steps: int = 0) -> Sampler:
    """Defaults are the constants baked into the reference graphs
    (t2s_stage_decoder_fp32.onnx#1780-1790, Inference.py:95)."""
    return Sampler(top_k, temperature, repetition_penalty, int(greedy), seed, max_steps, force_steps)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise EngineError(f"{_LIB_PATH} missing: build it with `python -m genie_tts_amd.build`")
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, i64p = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)
        L.gsv_last_error.restype = ctypes.c_char_p
        L.gsv_version.restype = ctypes.c_char_p
        if b"no packed-fp32" not in L.gsv_version():
            # built without build.py's NO_PACKED_FP32: its packed-FP32 ops can return 0 in lanes
            # 48-63 beside MFMA-heavy waves
            raise EngineError(f"{_LIB_PATH} was built with packed-FP32 ops: rebuild with "
                              "`python -m genie_tts_amd.build`")
        L.gsv_engine_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.gsv_engine_destroy.argtypes = [vp]
        L.gsv_set_weight.argtypes = [vp, ctypes.c_char_p, vp, ctypes.c_int, i64p, ctypes.c_int]
        L.gsv_finalize_weights.argtypes = [vp]
        L.gsv_reserve.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.gsv_t2s_encode.argtypes = [vp, ctypes.POINTER(Utt), vp, vp, vp]
        L.gsv_t2s_generate.argtypes = [vp, ctypes.c_int, ctypes.POINTER(Utt), ctypes.POINTER(Sampler),
                                       vp, i32, vp, vp]
        L.gsv_t2s_prefill.argtypes = [vp, ctypes.c_int, vp, i32, vp, i32, ctypes.POINTER(Sampler),
                                      vp, vp, vp]
        L.gsv_t2s_decode_steps.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Sampler),
                                           vp, vp, vp, vp]
        L.gsv_t2s_read_kv.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp,
                                      ctypes.POINTER(ctypes.c_int32), vp]
        L.gsv_vits_decode.argtypes = [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp, ctypes.c_float, vp, vp]
        L.gsv_vits_decode_batch.argtypes = [vp, i32, ctypes.POINTER(VitsItem), ctypes.c_float, vp]
        L.gsv_vits_decode_async.argtypes = [vp, ctypes.POINTER(VitsItem), ctypes.c_float, vp]
        L.gsv_vits_wait.argtypes = [vp, vp]
        L.gsv_vits_decode_batch_async.argtypes = [vp, i32, ctypes.POINTER(VitsItem), ctypes.c_float, vp]
        L.gsv_vits_batch_wait.argtypes = [vp, vp]
        L.gsv_t2s_prefetch.argtypes = [vp, ctypes.POINTER(Utt), ctypes.POINTER(Sampler), vp]
        L.gsv_t2s_generate_start.argtypes = [vp, ctypes.POINTER(Utt), ctypes.POINTER(Sampler), vp]
        L.gsv_t2s_generate_finish.argtypes = [vp, vp, i32, vp, vp]
        L.gsv_prompt_encode.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.gsv_ref_encode.argtypes = [vp, vp, i32, vp, vp]
        L.gsv_debug_copy.argtypes = [vp, ctypes.c_char_p, vp, ctypes.c_int64, vp]
        L.gsv_debug_conv1d.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_float, vp, ctypes.c_int64, vp]
        L.gsv_debug_conv1d_h.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_float, vp, vp]
        L.gsv_debug_ktrace.argtypes = [vp, vp, ctypes.c_int]
        L.gsv_debug_sample.argtypes = [vp, vp, ctypes.c_int, ctypes.POINTER(Sampler), ctypes.c_int, vp, vp, vp]
        L.gsv_probe.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_float), vp]
        L.gsv_set_timing.argtypes = [vp, ctypes.c_int]
        L.gsv_get_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
        L.gsv_get_kernel_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32)]
        L.gsv_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int]
        L.gsv_debug_ptrace.argtypes = [vp, vp, ctypes.c_int]
        L.gsv_get_counter.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
        L.gsv_hubert_frames.argtypes = [ctypes.c_int32]
        L.gsv_hubert.argtypes = [vp, vp, ctypes.c_int32, vp, vp]
        L.gsv_sv_frames.argtypes = [ctypes.c_int32]
        L.gsv_sv.argtypes = [vp, vp, ctypes.c_int32, vp, vp]
        L.gsv_roberta.argtypes = [vp, vp, vp, ctypes.c_int32, vp, ctypes.c_int32, vp, vp]
        L.gsv_roberta_batch.argtypes = [vp, ctypes.c_int32, vp, vp, vp, vp, vp, vp]
        L.gsv_f16_exact.argtypes = [vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        L.gsv_request_stop.argtypes = [vp, ctypes.c_int32]
        L.gsv_debug_hbm_copy.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp, ctypes.POINTER(ctypes.c_float)]
        _lib = L
    return _lib


EXPORTED = (
    "gsv_last_error", "gsv_version", "gsv_engine_create", "gsv_engine_destroy", "gsv_set_weight",
    "gsv_finalize_weights", "gsv_reserve", "gsv_t2s_encode", "gsv_t2s_generate", "gsv_t2s_prefill",
    "gsv_t2s_decode_steps", "gsv_t2s_read_kv", "gsv_vits_decode", "gsv_prompt_encode",
    "gsv_set_timing", "gsv_get_timing", "gsv_debug_copy", "gsv_debug_conv1d",
    "gsv_probe", "gsv_get_kernel_timing", "gsv_debug_sample", "gsv_debug_ktrace",
    "gsv_set_option", "gsv_debug_ptrace", "gsv_debug_conv1d_h", "gsv_vits_decode_batch",
    "gsv_get_counter", "gsv_hubert", "gsv_hubert_frames", "gsv_sv", "gsv_sv_frames", "gsv_roberta",
    "gsv_vits_decode_async",
    "gsv_vits_wait", "gsv_t2s_prefetch", "gsv_t2s_generate_start", "gsv_t2s_generate_finish",
    "gsv_vits_decode_batch_async", "gsv_vits_batch_wait", "gsv_ref_encode", "gsv_roberta_batch",
    "gsv_f16_exact", "gsv_request_stop", "gsv_debug_hbm_copy",
)


def hbm_copy_ms(src, dst, iters: int = 10) -> float:
    """Mean time of one float4 grid-stride device copy src -> dst (torch tensors, same byte
    size), the achievable-HBM probe of bench.py (gsv_debug_hbm_copy)."""
    import torch
    ms = ctypes.c_float(0.0)
    nbytes = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == nbytes and src.is_cuda and dst.is_cuda
    st = torch.cuda.current_stream(src.device).cuda_stream
    _check(lib().gsv_debug_hbm_copy(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), nbytes,
                                    iters, ctypes.c_void_p(st), ctypes.byref(ms)), "hbm copy probe")
    return float(ms.value)


def f16_exact(values) -> int:
    """gsv_f16_exact: -1 when every value is exactly an fp16 number (what the engine's
    fp16-only weight paths require), else the index of the first one that is not.
    A host-only check: needs the library, not a GPU."""
    import numpy as np
    v = np.ascontiguousarray(values, np.float32).reshape(-1)
    bad = ctypes.c_int64(0)
    rc = lib().gsv_f16_exact(v.ctypes.data_as(ctypes.c_void_p), v.size, ctypes.byref(bad))
    if rc < 0:
        _check(rc, "gsv_f16_exact")
    return int(bad.value)


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().gsv_last_error().decode(errors="replace")
        if rc == GSV_E_STOPPED:
            raise EngineStopped(f"{what}: {msg}")
        raise EngineError(f"{what} failed ({rc}): {msg}")


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise EngineError("no HIP device visible: the MI355X engine has no CPU fallback")
    return torch


def _stream():
    return ctypes.c_void_p(_torch().cuda.current_stream().cuda_stream)


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def debug_conv1d(x, w, bias=None, dil=1, pad=0, in_act=False, slope=0.1, splitk_ws=None):
    """Run the engine's conv1d kernel once (tests): x [Cin,T], w [Cout,Cin,K] cuda fp32.
    splitk_ws (cuda fp32 tensor) enables the split-K path for small grids."""
    torch = _torch()
    cin, tin = x.shape
    cout, _, k = w.shape
    tout = tin + 2 * pad - dil * (k - 1)
    out = torch.empty((cout, tout), dtype=torch.float32, device=x.device)
    _check(lib().gsv_debug_conv1d(_ptr(x), cin, tin, _ptr(w), cout, k, dil, pad, _ptr(bias), _ptr(out),
                                  tout, int(in_act), ctypes.c_float(slope), _ptr(splitk_ws),
                                  0 if splitk_ws is None else splitk_ws.numel(), _stream()), "gsv_debug_conv1d")
    return out


def debug_conv1d_h(x, v, scale, bias=None, dil=1, pad=0, in_act=False, slope=0.1):
    """Run the f16-split MFMA conv once (tests): x [Cin,T] cuda fp32, v [Cout,Cin,K] fp16-valued,
    scale [Cout] (weight = v * scale).  Returns (out, overflow flag)."""
    torch = _torch()
    cin, tin = x.shape
    cout, _, k = v.shape
    tout = tin + 2 * pad - dil * (k - 1)
    wh = v.to(torch.float16).permute(0, 2, 1).contiguous().to(x.device)     # [Cout][K][Cin]
    sc = scale.to(torch.float32).contiguous().to(x.device)
    out = torch.empty((cout, tout), dtype=torch.float32, device=x.device)
    ovf = torch.zeros(1, dtype=torch.int32, device=x.device)
    _check(lib().gsv_debug_conv1d_h(_ptr(x), cin, tin, _ptr(wh), _ptr(sc), cout, k, dil, pad, _ptr(bias), _ptr(out),
                                    tout, int(in_act), ctypes.c_float(slope), _ptr(ovf), _stream()),
           "gsv_debug_conv1d_h")
    return out, int(ovf.item())


def debug_sample(logits, seen, sampler: "Sampler", step: int):
    """Run the decode sampler kernel (tests): logits [B,1025] cuda f32, seen [B,33] cuda int32 bitmaps."""
    torch = _torch()
    B = logits.shape[0]
    tok = torch.empty((B,), dtype=torch.int64, device=logits.device)
    stop = torch.empty((B,), dtype=torch.uint8, device=logits.device)
    _check(lib().gsv_debug_sample(_ptr(logits), _ptr(seen), B, ctypes.byref(sampler), step, _ptr(tok), _ptr(stop),
                                  _stream()), "gsv_debug_sample")
    return tok, stop


class Engine:
    """One engine per GPU process, holding one character's weights."""

    def __init__(self, weights: Dict[str, Dict[str, np.ndarray]], version: str = "v2",
                 device: int = 0, pe_div_term: Optional[np.ndarray] = None):
        torch = _torch()
        self.torch = torch
        self.device = device
        self.version = version
        torch.cuda.set_device(device)
        h = ctypes.c_void_p()
        _check(lib().gsv_engine_create(device, GSV_V2 if version == "v2" else GSV_V2PP,
                                       ctypes.byref(h)), "gsv_engine_create")
        self.h = h
        for group in weights.values():
            for name, arr in group.items():
                self._set(name, arr)
        if pe_div_term is not None:
            self._set("pe.div_term", np.asarray(pe_div_term, np.float32))
        _check(lib().gsv_finalize_weights(self.h), "gsv_finalize_weights")
        self.dev = torch.device("cuda", device)
        with _engines_lock:
            _engines.add(self)
            if _stop_on:
                lib().gsv_request_stop(self.h, 1)

    def request_stop(self, on: bool = True):
        """gsv_request_stop: while set, T2S generates raise EngineStopped (a running decode
        leaves within two loop steps).  Callable from another thread."""
        _check(lib().gsv_request_stop(self.h, int(on)), "gsv_request_stop")

    def _set(self, name: str, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        if a.dtype == np.float16:
            dt = GSV_F16
        else:
            a = np.ascontiguousarray(a, dtype=np.float32)
            dt = GSV_F32
        dims = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
        _check(lib().gsv_set_weight(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), dt,
                                    dims, a.ndim), f"gsv_set_weight({name})")

    def close(self):
        if getattr(self, "h", None):
            lib().gsv_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- helpers
    def _dev(self, x, dtype):
        t = self.torch
        if x is None:
            return None
        if isinstance(x, t.Tensor):
            return x.to(device=self.dev, dtype=dtype).contiguous()
        return t.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=self.dev).contiguous()

    def make_utt(self, ref_seq, text_seq, ref_bert, text_bert, ssl, force_steps: int = 0):
        t = self.torch
        flat = lambda a: a.reshape(-1) if isinstance(a, t.Tensor) else np.asarray(a).reshape(-1)
        keep = [self._dev(flat(ref_seq), t.int64),
                self._dev(flat(text_seq), t.int64),
                None if ref_bert is None else self._dev(ref_bert, t.float32),
                None if text_bert is None else self._dev(text_bert, t.float32),
                self._dev(ssl, t.float32).reshape(768, -1)]
        u = Utt(keep[0].data_ptr(), keep[0].numel(), keep[1].data_ptr(), keep[1].numel(),
                0 if keep[2] is None else keep[2].data_ptr(),
                0 if keep[3] is None else keep[3].data_ptr(),
                keep[4].data_ptr(), keep[4].shape[1], int(force_steps))
        return u, keep

    def reserve(self, batch: int, tokens: int):
        _check(lib().gsv_reserve(self.h, batch, tokens), "gsv_reserve")

    # -------------------------------------------------------------- T2S
    def t2s_encode(self, ref_seq, text_seq, ref_bert, text_bert, ssl):
        t = self.torch
        u, keep = self.make_utt(ref_seq, text_seq, ref_bert, text_bert, ssl)
        L = u.n_ref + u.n_text
        x = t.empty((L, 512), dtype=t.float32, device=self.dev)
        prompts = t.empty((u.n_ssl // 2,), dtype=t.int64, device=self.dev)
        _check(lib().gsv_t2s_encode(self.h, ctypes.byref(u), _ptr(x), _ptr(prompts), _stream()),
               "gsv_t2s_encode")
        return x, prompts

    def t2s_generate(self, utts: Sequence[Tuple], sampler: Optional[Sampler] = None,
                     out_stride: int = 1024) -> List[np.ndarray]:
        """utts: sequence of (ref_seq, text_seq, ref_bert, text_bert, ssl[, force_steps]);
        force_steps > 0 runs that utterance for exactly that many loop steps (EOS ignored)."""
        if len(utts) > MAX_BATCH:   # the engine decodes up to 64 sequences together
            out = []
            for i in range(0, len(utts), MAX_BATCH):
                out += self.t2s_generate(utts[i:i + MAX_BATCH], sampler, out_stride)
            return out
        arr = (Utt * len(utts))()
        keep = []
        pf = getattr(self, "_pf", [])
        hit = next((j for j, p in enumerate(pf) if len(utts) == 1 and p[0] is utts[0]), None)
        # consumed entries go; on a single-utterance miss the engine keeps a queued
        # prefetch (the latest), whose buffers must stay alive; a batch drops all
        self._pf = pf[hit + 1:] if hit is not None else pf[-1:] if len(utts) == 1 else []
        for i, u in enumerate(utts):
            if hit is not None:
                arr[i], k = pf[hit][1], pf[hit][2]   # the prefetched utterance: the same device buffers
            else:
                arr[i], k = self.make_utt(*u)
            keep.append(k)
        sp = sampler or make_sampler()
        out = np.zeros((len(utts), out_stride), dtype=np.int64)
        lens = np.zeros(len(utts), dtype=np.int32)
        _check(lib().gsv_t2s_generate(self.h, len(utts), arr, ctypes.byref(sp),
                                      out.ctypes.data_as(ctypes.c_void_p), out_stride,
                                      lens.ctypes.data_as(ctypes.c_void_p), _stream()),
               "gsv_t2s_generate")
        return [out[i, :lens[i]].copy() for i in range(len(utts))]

    def t2s_prefetch(self, utt: Tuple, sampler: Optional[Sampler] = None):
        """Encode + prefill `utt` (a t2s_generate tuple) ahead on the vocoder CUs while the
        current decode runs (gsv_t2s_prefetch); the next t2s_generate([utt], sampler)
        with this same tuple object decodes from it."""
        u, keep = self.make_utt(*utt)
        sp = sampler or make_sampler()
        _check(lib().gsv_t2s_prefetch(self.h, ctypes.byref(u), ctypes.byref(sp), _stream()), "gsv_t2s_prefetch")
        # the engine holds a launched prefetch (for the next generate) and a queued one
        self._pf = (getattr(self, "_pf", []) + [(utt, u, keep)])[-2:]

    def t2s_generate_start(self, utt: Tuple, sampler: Optional[Sampler] = None):
        """Queue the T2S of one utterance (gsv_t2s_generate_start) and return at once;
        up to two in flight, so the next decode is queued behind the running one.
        t2s_generate_finish() returns the oldest one's tokens."""
        pf = getattr(self, "_pf", [])
        hit = next((j for j, p in enumerate(pf) if p[0] is utt), None)
        if hit is not None:
            u, keep = pf[hit][1], pf[hit][2]
            self._pf = pf[hit + 1:]
        else:
            u, keep = self.make_utt(*utt)
            self._pf = pf[-1:]
        sp = sampler or make_sampler()
        _check(lib().gsv_t2s_generate_start(self.h, ctypes.byref(u), ctypes.byref(sp), _stream()),
               "gsv_t2s_generate_start")
        if not hasattr(self, "_gq"):
            self._gq = []
        self._gq.append((u, keep))

    def t2s_generate_finish(self, out_stride: int = 1024) -> np.ndarray:
        """Tokens of the oldest started generate (trimmed, EOS-filtered)."""
        out = np.zeros((out_stride,), dtype=np.int64)
        n = np.zeros(1, dtype=np.int32)
        try:
            _check(lib().gsv_t2s_generate_finish(self.h, out.ctypes.data_as(ctypes.c_void_p), out_stride,
                                                 n.ctypes.data_as(ctypes.c_void_p), _stream()),
                   "gsv_t2s_generate_finish")
        finally:
            if getattr(self, "_gq", None):
                self._gq.pop(0)
        return out[:n[0]].copy()

    def t2s_prefill(self, x, prompts, sampler: Optional[Sampler] = None, seq: int = 0):
        t = self.torch
        x = self._dev(x, t.float32).reshape(-1, 512)
        prompts = self._dev(np.asarray(prompts).reshape(-1) if not isinstance(prompts, t.Tensor)
                            else prompts.reshape(-1), t.int64)
        L, P = x.shape[0], prompts.numel()
        self.reserve(max(1, seq + 1), L + P + 520)
        y = t.empty((P + 1,), dtype=t.int64, device=self.dev)
        logits = t.empty((1025,), dtype=t.float32, device=self.dev)
        sp = sampler or make_sampler()
        _check(lib().gsv_t2s_prefill(self.h, seq, _ptr(x), L, _ptr(prompts), P, ctypes.byref(sp),
                                     _ptr(y), _ptr(logits), _stream()), "gsv_t2s_prefill")
        return y, logits

    def t2s_decode_steps(self, steps: int, sampler: Optional[Sampler] = None, y_cap: int = 4096):
        t = self.torch
        y = t.empty((y_cap,), dtype=t.int64, device=self.dev)
        stop = t.empty((steps,), dtype=t.uint8, device=self.dev)
        logits = t.empty((steps, 1025), dtype=t.float32, device=self.dev)
        sp = sampler or make_sampler()
        _check(lib().gsv_t2s_decode_steps(self.h, 0, steps, ctypes.byref(sp), _ptr(y), _ptr(stop),
                                          _ptr(logits), _stream()), "gsv_t2s_decode_steps")
        return y, stop, logits

    def t2s_read_kv(self, layer: int, seq: int = 0, cap: int = 4096):
        t = self.torch
        k = t.empty((cap, 512), dtype=t.float32, device=self.dev)
        v = t.empty((cap, 512), dtype=t.float32, device=self.dev)
        n = ctypes.c_int32()
        _check(lib().gsv_t2s_read_kv(self.h, seq, layer, _ptr(k), _ptr(v), ctypes.byref(n),
                                     _stream()), "gsv_t2s_read_kv")
        return k[:n.value], v[:n.value]

    # -------------------------------------------------------------- VITS
    def _ids(self, x):
        t = self.torch
        return self._dev(np.asarray(x).reshape(-1) if not isinstance(x, t.Tensor) else x.reshape(-1), t.int64)

    def vits_decode(self, text_seq, pred_semantic, ref_audio=None, ge=None, ge_advanced=None,
                    eps=None, noise_scale: float = 0.5, noise_seed: Optional[int] = None):
        """vits_fp32.onnx for one utterance.  Noise of z_p: eps (tensor/array [192, 2G]) if
        given, else the engine's Philox N(0,1) stream keyed by noise_seed if given, else zeros."""
        if noise_seed is not None and eps is None:
            return self.vits_decode_batch([dict(text_seq=text_seq, pred_semantic=pred_semantic, ref_audio=ref_audio,
                                                ge=ge, ge_advanced=ge_advanced, noise_seed=noise_seed)],
                                          noise_scale)[0]
        t = self.torch
        ts = self._ids(text_seq)
        sem = self._ids(pred_semantic)
        G = sem.numel()
        ra = None if ref_audio is None else self._dev(ref_audio, t.float32).reshape(-1)
        g = None if ge is None else self._dev(ge, t.float32).reshape(-1)
        ga = None if ge_advanced is None else self._dev(ge_advanced, t.float32).reshape(-1)
        e = None if eps is None else self._dev(eps, t.float32).reshape(192, 2 * G)
        audio = t.empty((1280 * G,), dtype=t.float32, device=self.dev)
        _check(lib().gsv_vits_decode(self.h, _ptr(ts), ts.numel(), _ptr(sem), G, _ptr(ra),
                                     0 if ra is None else ra.numel(), _ptr(g), _ptr(ga), _ptr(e),
                                     ctypes.c_float(noise_scale), _ptr(audio), _stream()),
               "gsv_vits_decode")
        return audio

    def _vits_item(self, it: dict):
        """(VitsItem, tensors it points at, audio tensor) of one vocoder call."""
        t = self.torch
        ts, sem = self._ids(it["text_seq"]), self._ids(it["pred_semantic"])
        G = sem.numel()
        ra = it.get("ref_audio")
        ra = None if ra is None else self._dev(ra, t.float32).reshape(-1)
        g = it.get("ge")
        g = None if g is None else self._dev(g, t.float32).reshape(-1)
        ga = it.get("ge_advanced")
        ga = None if ga is None else self._dev(ga, t.float32).reshape(-1)
        e = it.get("eps")
        e = None if e is None else self._dev(e, t.float32).reshape(192, 2 * G)
        seed = it.get("noise_seed")
        mode = 1 if e is not None else (2 if seed is not None else 0)
        audio = t.empty((1280 * G,), dtype=t.float32, device=self.dev)
        item = VitsItem(ts.data_ptr(), ts.numel(), sem.data_ptr(), G, 0 if ra is None else ra.data_ptr(),
                        0 if ra is None else ra.numel(), 0 if g is None else g.data_ptr(),
                        0 if ga is None else ga.data_ptr(), 0 if e is None else e.data_ptr(),
                        int(seed or 0) & 0xFFFFFFFFFFFFFFFF, mode, audio.data_ptr())
        return item, [ts, sem, ra, g, ga, e], audio

    def vits_decode_batch(self, items: Sequence[dict], noise_scale: float = 0.5):
        """Several vocoder calls at once (concurrent engine lanes).  Each item: text_seq,
        pred_semantic, and ref_audio (V2) or ge + ge_advanced (V2ProPlus); optional eps or
        noise_seed.  Returns one audio tensor [1280 G] per item."""
        arr = (VitsItem * len(items))()
        keep, outs = [], []
        for i, it in enumerate(items):
            arr[i], k, audio = self._vits_item(it)
            keep += k
            outs.append(audio)
        _check(lib().gsv_vits_decode_batch(self.h, len(items), arr, ctypes.c_float(noise_scale), _stream()),
               "gsv_vits_decode_batch")
        return outs

    def vits_decode_batch_async(self, items: Sequence[dict], noise_scale: float = 0.5):
        """vits_decode_batch without the join (gsv_vits_decode_batch_async): the lanes run
        beside whatever T2S is issued next.  Returns the audio tensors, valid after
        vits_batch_wait()."""
        arr = (VitsItem * len(items))()
        keep, outs = [], []
        for i, it in enumerate(items):
            arr[i], k, audio = self._vits_item(it)
            keep += k
            outs.append(audio)
        _check(lib().gsv_vits_decode_batch_async(self.h, len(items), arr, ctypes.c_float(noise_scale),
                                                 _stream()), "gsv_vits_decode_batch_async")
        # items and device buffers live until the wait -- also a previous batch's, which this
        # call only ordered behind the engine stream (its lanes may still read them)
        # (one generation back: a batch older than the previous one was joined by this launch)
        prev = getattr(self, "_vits_batch_keep", None)
        self._vits_batch_keep = (arr, keep, outs, prev[:3] if prev else None)
        return outs

    def vits_batch_wait(self):
        """Finish the pending vits_decode_batch_async; orders the current stream after it."""
        _check(lib().gsv_vits_batch_wait(self.h, _stream()), "gsv_vits_batch_wait")
        self._vits_batch_keep = None

    vocoder_cus = 0

    def set_vocoder_cus(self, k: int):
        """Reserve k CUs for the overlapped vocoder (0: off; see gsv_vits_decode_async)."""
        self.set_option("vocoder_cus", k)
        self.vocoder_cus = int(k)

    def vits_decode_async(self, item: dict, noise_scale: float = 0.5):
        """Start one vocoder call on the vocoder CUs (gsv_vits_decode_async) and return its
        audio tensor [1280 G], valid after vits_wait().  item as for vits_decode_batch."""
        it, keep, audio = self._vits_item(item)
        _check(lib().gsv_vits_decode_async(self.h, ctypes.byref(it), ctypes.c_float(noise_scale), _stream()),
               "gsv_vits_decode_async")
        self._vits_keep = keep   # device inputs stay alive until the call is finished
        return audio

    def vits_wait(self):
        """Finish the pending vits_decode_async call; orders the current stream after it."""
        _check(lib().gsv_vits_wait(self.h, _stream()), "gsv_vits_wait")
        self._vits_keep = None

    def ref_encode(self, ref_audio):
        """V2: the vocoder's reference branch alone (gsv_ref_encode) -> ge [512] on the device;
        pass it as ge= (without ref_audio) to every vocoder call against this reference."""
        t = self.torch
        ra = self._dev(ref_audio, t.float32).reshape(-1)
        ge = t.empty((512,), dtype=t.float32, device=self.dev)
        _check(lib().gsv_ref_encode(self.h, _ptr(ra), ra.numel(), _ptr(ge), _stream()), "gsv_ref_encode")
        return ge

    def prompt_encode(self, ref_audio, sv_emb):
        t = self.torch
        ra = self._dev(ref_audio, t.float32).reshape(-1)
        sv = self._dev(sv_emb, t.float32).reshape(-1)
        ge = t.empty((1024,), dtype=t.float32, device=self.dev)
        ga = t.empty((512,), dtype=t.float32, device=self.dev)
        _check(lib().gsv_prompt_encode(self.h, _ptr(ra), ra.numel(), _ptr(sv), _ptr(ge), _ptr(ga),
                                       _stream()), "gsv_prompt_encode")
        return ge, ga

    def hubert(self, audio_16k):
        """CN-HuBERT (gsv_hubert): raw 16 kHz audio [N] -> ssl_content [768, T] on the device."""
        t = self.torch
        a = self._dev(audio_16k, t.float32).reshape(-1)
        T = lib().gsv_hubert_frames(a.numel())
        if T < 1:
            raise EngineError(f"audio of {a.numel()} samples is too short for CN-HuBERT")
        out = t.empty((768, T), dtype=t.float32, device=self.dev)
        _check(lib().gsv_hubert(self.h, _ptr(a), a.numel(), _ptr(out), _stream()), "gsv_hubert")
        return out

    def sv(self, audio_16k):
        """Speaker verification (gsv_sv): 16 kHz audio [N] -> sv_emb [1, 20480] on the device."""
        t = self.torch
        a = self._dev(audio_16k, t.float32).reshape(-1)
        if lib().gsv_sv_frames(a.numel()) < 1:
            raise EngineError(f"audio of {a.numel()} samples is too short for the SV fbank (400 needed)")
        out = t.empty((1, 20480), dtype=t.float32, device=self.dev)
        _check(lib().gsv_sv(self.h, _ptr(a), a.numel(), _ptr(out), _stream()), "gsv_sv")
        return out

    def roberta(self, input_ids, repeats, attention_mask=None):
        """RoBERTa (gsv_roberta): token ids [N] (CLS .. SEP), word2ph [n_chars] ->
        text_bert [sum(word2ph), 1024] on the device."""
        t = self.torch
        ids = self._dev(np.asarray(input_ids).reshape(-1) if not isinstance(input_ids, t.Tensor)
                        else input_ids.reshape(-1), t.int64)
        rep = np.ascontiguousarray(np.asarray(repeats, np.int64).reshape(-1))
        mask = None if attention_mask is None else np.ascontiguousarray(np.asarray(attention_mask, np.int64).reshape(-1))
        out = t.empty((int(rep.sum()), 1024), dtype=t.float32, device=self.dev)
        _check(lib().gsv_roberta(self.h, _ptr(ids), None if mask is None else mask.ctypes.data_as(ctypes.c_void_p),
                                 ids.numel(), rep.ctypes.data_as(ctypes.c_void_p), rep.size, _ptr(out), _stream()),
               "gsv_roberta")
        return out

    def roberta_batch(self, sentences):
        """Packed RoBERTa over several sentences (gsv_roberta_batch): sentences = [(input_ids
        [N_i] CLS .. SEP, word2ph [C_i])] -> one text_bert tensor [sum(word2ph_i), 1024] per
        sentence (views of one device buffer), identical to per-sentence roberta()."""
        t = self.torch
        ids = [self._ids(i) for i, _ in sentences]          # host arrays or device tensors
        reps = [np.asarray(r, np.int64).reshape(-1) for _, r in sentences]
        dids = t.cat(ids) if len(ids) > 1 else ids[0]
        nt = np.asarray([i.numel() for i in ids], np.int32)
        nc = np.asarray([r.size for r in reps], np.int32)
        rep = np.ascontiguousarray(np.concatenate(reps)) if sum(r.size for r in reps) else np.zeros(1, np.int64)
        rows = [int(r.sum()) for r in reps]
        out = t.empty((max(1, sum(rows)), 1024), dtype=t.float32, device=self.dev)
        _check(lib().gsv_roberta_batch(self.h, len(sentences), _ptr(dids), nt.ctypes.data_as(ctypes.c_void_p),
                                       rep.ctypes.data_as(ctypes.c_void_p), nc.ctypes.data_as(ctypes.c_void_p),
                                       _ptr(out), _stream()), "gsv_roberta_batch")
        offs = np.concatenate([[0], np.cumsum(rows)])
        return [out[offs[i]:offs[i + 1]] for i in range(len(sentences))]

    def debug_copy(self, name: str, n: int):
        t = self.torch
        out = t.empty((n,), dtype=t.float32, device=self.dev)
        _check(lib().gsv_debug_copy(self.h, name.encode(), _ptr(out), n, _stream()), "gsv_debug_copy")
        return out

    def probe(self, which: int, batch: int = 1, iters: int = 200) -> float:
        """Average microseconds per launch of one kernel configuration (see gsv_probe)."""
        us = ctypes.c_float()
        _check(lib().gsv_probe(self.h, which, batch, iters, ctypes.byref(us), _stream()), "gsv_probe")
        return us.value

    def set_timing(self, on: bool = True):
        _check(lib().gsv_set_timing(self.h, int(on)), "gsv_set_timing")

    def kernel_timing(self):
        """(average microseconds, samples) of the live-sampled dominant decode kernel."""
        us, n = ctypes.c_float(), ctypes.c_int32()
        _check(lib().gsv_get_kernel_timing(self.h, ctypes.byref(us), ctypes.byref(n)), "gsv_get_kernel_timing")
        return us.value, n.value

    def set_option(self, name: str, value: int):
        """Engine option (see gsv_set_option): "persist" decode path, "ptrace" phase stamps."""
        _check(lib().gsv_set_option(self.h, name.encode(), int(value)), "gsv_set_option")

    def counter(self, name: str) -> int:
        """Engine counter (gsv_get_counter): persist_timeouts, persist1_f16_reruns, vits_f32_reruns,
        sv_f32_reruns, w16_split_tensors, persist_disabled (timeout back-off holds begun),
        persist_launches, persist_hold (generates left in the current hold), stops, graph_fallbacks,
        retired_bytes (replaced device buffers not yet freed), reclaimed_bytes, reclaims."""
        v = ctypes.c_int64()
        _check(lib().gsv_get_counter(self.h, name.encode(), ctypes.byref(v)), "gsv_get_counter")
        return v.value

    def ptrace(self) -> np.ndarray:
        """[256 workgroups][16 slots] stamps of the persistent decode (option ptrace):
        slots 0-7 the 100 MHz clock, 8-15 the shader clock at the same points."""
        out = np.zeros((256, 16), np.uint64)
        _check(lib().gsv_debug_ptrace(self.h, out.ctypes.data_as(ctypes.c_void_p), out.size), "gsv_debug_ptrace")
        return out

    def ktrace(self) -> np.ndarray:
        """[3 kernels][256 blocks][8 slots] realtime stamps (GENIE_KTRACE=1 builds only)."""
        out = np.zeros((3, 256, 8), np.uint64)
        _check(lib().gsv_debug_ktrace(self.h, out.ctypes.data_as(ctypes.c_void_p), out.size), "gsv_debug_ktrace")
        return out

    def timing(self) -> List[float]:
        a = (ctypes.c_float * 4)()
        _check(lib().gsv_get_timing(self.h, a), "gsv_get_timing")
        return list(a)
