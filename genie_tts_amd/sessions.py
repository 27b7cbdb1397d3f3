"""InferenceSession-shaped objects backed by the MI355X engine.

The reference drives five onnxruntime sessions per character through
`session.run(output_names, input_feed) -> list[np.ndarray]` and, for the stage
decoder, `session.get_inputs()` (src/genie_tts/Core/Inference.py:47,55,76,88,93,102;
src/genie_tts/Audio/ReferenceAudio.py:73).  These classes keep that contract --
same input/output names, dtypes and shapes as the graph templates (SURVEY.md
Appendix A), caller-owned numpy outputs, exceptions on error -- so the
reference's own `GENIE.t2s_cpu` loop runs unchanged on top of them.

All sessions of one character share one `Engine` (device weights, KV cache).
The T2S decoder keeps its KV cache on the device: the `present_*` outputs are
read back only because the session contract returns them; a stage-decoder call
must continue the sequence the previous first-stage/stage call produced (the
only way the reference uses it, Inference.py:95-103), otherwise
`SessionStateError` is raised -- the device cache cannot be re-seeded from host
arrays.  The fast path that skips all of this is `inference.GENIE.t2s` (one
`gsv_t2s_generate` call).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .engine import Engine, make_sampler

N_LAYERS = 24


class SessionStateError(RuntimeError):
    pass


@dataclass(frozen=True)
class NodeArg:
    """Stand-in for onnxruntime.NodeArg (name/shape/type as the templates declare)."""
    name: str
    shape: tuple
    type: str


def _kv_names(prefix: str) -> List[str]:
    out = []
    for l in range(N_LAYERS):
        out += [f"{prefix}_k_layer_{l}", f"{prefix}_v_layer_{l}"]
    return out


class _Session:
    INPUTS: Sequence[NodeArg] = ()
    OUTPUTS: Sequence[NodeArg] = ()

    def __init__(self, engine: Engine):
        self.engine = engine

    def get_inputs(self) -> List[NodeArg]:
        return list(self.INPUTS)

    def get_outputs(self) -> List[NodeArg]:
        return list(self.OUTPUTS)

    def _select(self, output_names, outs: Dict[str, np.ndarray]) -> List[np.ndarray]:
        names = [o.name for o in self.OUTPUTS] if output_names is None else list(output_names)
        missing = [n for n in names if n not in outs]
        if missing:
            raise KeyError(f"unknown output(s) {missing}")
        return [outs[n] for n in names]

    @staticmethod
    def _need(feed, *names):
        missing = [n for n in names if n not in feed]
        if missing:
            raise KeyError(f"missing input(s) {missing}")


def _np(t) -> np.ndarray:
    return t.detach().cpu().numpy()


class EncoderSession(_Session):
    """t2s_encoder_fp32.onnx (reference call: Inference.py:76-85)."""
    INPUTS = (NodeArg("ref_seq", (1, "R"), "tensor(int64)"), NodeArg("text_seq", (1, "S"), "tensor(int64)"),
              NodeArg("ref_bert", ("R", 1024), "tensor(float)"), NodeArg("text_bert", ("S", 1024), "tensor(float)"),
              NodeArg("ssl_content", (1, 768, "H"), "tensor(float)"))
    OUTPUTS = (NodeArg("x", (1, "L", 512), "tensor(float)"), NodeArg("prompts", (1, "P"), "tensor(int64)"))

    def run(self, output_names, input_feed):
        self._need(input_feed, "ref_seq", "text_seq", "ref_bert", "text_bert", "ssl_content")
        f = input_feed
        x, prompts = self.engine.t2s_encode(f["ref_seq"], f["text_seq"], f["ref_bert"], f["text_bert"],
                                            np.asarray(f["ssl_content"], np.float32).reshape(768, -1))
        return self._select(output_names, {"x": _np(x)[None], "prompts": _np(prompts)[None]})


class _T2SState:
    """Host mirror of the device slot: the y the device holds, for continuity checks."""

    def __init__(self):
        self.y: Optional[np.ndarray] = None


class _DecoderBase(_Session):
    def __init__(self, engine: Engine, emb: np.ndarray, state: _T2SState):
        super().__init__(engine)
        self.emb = emb            # ar_audio_embedding table (y_emb = emb[y[:-1]])
        self.state = state

    def _outs(self, y: np.ndarray, with_kv: bool) -> Dict[str, np.ndarray]:
        outs = {"y": y[None].astype(np.int64), "y_emb": self.emb[y[:-1]][None].astype(np.float32)}
        if with_kv:
            for l in range(N_LAYERS):
                k, v = self.engine.t2s_read_kv(l)
                outs[f"present_k_layer_{l}"] = _np(k)[:, None, :]
                outs[f"present_v_layer_{l}"] = _np(v)[:, None, :]
        return outs

    def _wants_kv(self, output_names) -> bool:
        return output_names is None or any(str(n).startswith("present_") for n in output_names)


class FirstStageDecoderSession(_DecoderBase):
    """t2s_first_stage_decoder_fp32.onnx (reference call: Inference.py:88-90)."""
    INPUTS = (NodeArg("x", (1, "L", 512), "tensor(float)"), NodeArg("prompts", (1, "P"), "tensor(int64)"))
    OUTPUTS = (NodeArg("y", (1, "P+1"), "tensor(int64)"), NodeArg("y_emb", (1, "P", 512), "tensor(float)"),
               *[NodeArg(n, ("L+P", 1, 512), "tensor(float)") for n in _kv_names("present")])

    def __init__(self, engine, emb, state, sampler=None):
        super().__init__(engine, emb, state)
        self.sampler = sampler or make_sampler()

    def run(self, output_names, input_feed):
        self._need(input_feed, "x", "prompts")
        y, _ = self.engine.t2s_prefill(np.asarray(input_feed["x"], np.float32).reshape(-1, 512),
                                       np.asarray(input_feed["prompts"]).reshape(-1), self.sampler)
        yh = _np(y)
        self.state.y = yh.copy()
        return self._select(output_names, self._outs(yh, self._wants_kv(output_names)))


class StageDecoderSession(_DecoderBase):
    """t2s_stage_decoder_fp32.onnx (reference call: Inference.py:93-103), one step per run."""
    INPUTS = (NodeArg("iy", (1, "n"), "tensor(int64)"), NodeArg("iy_emb", (1, "n-1", 512), "tensor(float)"),
              *[NodeArg(n, ("T", 1, 512), "tensor(float)") for n in _kv_names("past")])
    OUTPUTS = (NodeArg("y", (1, "n+1"), "tensor(int64)"), NodeArg("y_emb", (1, "n", 512), "tensor(float)"),
               NodeArg("stop_condition_tensor", (), "tensor(bool)"),
               *[NodeArg(n, ("T+1", 1, 512), "tensor(float)") for n in _kv_names("present")])

    def __init__(self, engine, emb, state, sampler=None):
        super().__init__(engine, emb, state)
        self.sampler = sampler or make_sampler()

    def run(self, output_names, input_feed):
        self._need(input_feed, "iy")
        iy = np.asarray(input_feed["iy"]).reshape(-1)
        if self.state.y is None or iy.shape != self.state.y.shape or not np.array_equal(iy, self.state.y):
            raise SessionStateError("stage decoder input does not continue the device-resident sequence "
                                    "(run the first-stage decoder first and feed its outputs back)")
        y, stop, _ = self.engine.t2s_decode_steps(1, self.sampler)
        n = iy.size + 1
        yh = _np(y[:n])
        self.state.y = yh.copy()
        outs = self._outs(yh, self._wants_kv(output_names))
        outs["stop_condition_tensor"] = np.array(bool(_np(stop)[0]))
        return self._select(output_names, outs)


class VitsSession(_Session):
    """vits_fp32.onnx (reference calls: Inference.py:47-51 (V2), 55-60 (V2ProPlus)).

    z_p noise: the graph draws RandomNormalLike x noise_scale (0.5) on every call
    (vits(v2)#6490).  noise="philox" (default) draws it from the engine's device
    Philox N(0,1) stream, a fresh seed per call; noise="zero" is the deterministic
    test mode; `eps_fn(G) -> [192, 2G]` fixes it explicitly."""
    OUTPUTS = (NodeArg("audio", ("1280*G",), "tensor(float)"),)

    def __init__(self, engine, version: str, noise_scale: float = 0.5, eps_fn=None, noise: str = "philox",
                 seed: int = 0x5EED0000):
        super().__init__(engine)
        if noise not in ("philox", "zero"):
            raise ValueError("noise must be 'philox' or 'zero'")
        self.version = version
        self.noise_scale = noise_scale
        self.eps_fn = eps_fn
        self.noise = noise
        self._seed = seed
        common = (NodeArg("text_seq", (1, "S"), "tensor(int64)"), NodeArg("pred_semantic", (1, 1, "G"), "tensor(int64)"))
        self.INPUTS = common + ((NodeArg("ref_audio", (1, "N"), "tensor(float)"),) if version == "v2" else
                                (NodeArg("ge", (1, 1024, 1), "tensor(float)"),
                                 NodeArg("ge_advanced", (1, 512, 1), "tensor(float)")))

    _ref = _ref_key = _ref_ge = None

    def v2_cond(self, ref_audio) -> dict:
        """V2 conditioning of a vocoder call.  The graph recomputes the reference branch
        (refer spectrogram -> MelStyleEncoder -> ge, vits_fp32.onnx(v2)#79-271) on every
        run although it depends on the reference only; here it runs once per reference
        (gsv_ref_encode) and later calls pass ge -- identical audio.  A host array is
        recognised by identity plus a content fingerprint (so an array changed in place
        is re-encoded); device tensors are encoded per call."""
        if not isinstance(ref_audio, np.ndarray):
            return dict(ref_audio=ref_audio)
        a = np.ascontiguousarray(ref_audio, np.float32).reshape(-1)
        key = (a.shape, float(a.sum(dtype=np.float64)), a[:: max(1, a.size // 64)].tobytes())
        if self._ref is not ref_audio or self._ref_key != key:
            self._ref_ge = self.engine.ref_encode(a)
            self._ref, self._ref_key = ref_audio, key
        return dict(ge=self._ref_ge)

    def next_seed(self):
        """Seed of the next call's noise (None in zero mode)."""
        if self.noise == "zero":
            return None
        self._seed = (self._seed + 1) & 0xFFFFFFFFFFFFFFFF
        return self._seed

    def run(self, output_names, input_feed):
        f = input_feed
        self._need(f, "text_seq", "pred_semantic")
        sem = np.asarray(f["pred_semantic"]).reshape(-1)
        eps = self.eps_fn(sem.size) if self.eps_fn else None
        seed = None if eps is not None else self.next_seed()
        if self.version == "v2":
            self._need(f, "ref_audio")
            cond = self.v2_cond(f["ref_audio"])
        else:
            self._need(f, "ge", "ge_advanced")
            cond = dict(ge=f["ge"], ge_advanced=f["ge_advanced"])
        audio = self.engine.vits_decode(f["text_seq"], sem, eps=eps, noise_scale=self.noise_scale, noise_seed=seed,
                                        **cond)
        return self._select(output_names, {"audio": _np(audio)})


class PromptEncoderSession(_Session):
    """prompt_encoder_fp32.onnx, V2ProPlus (reference call: ReferenceAudio.py:73-76)."""
    INPUTS = (NodeArg("ref_audio", (1, "N"), "tensor(float)"), NodeArg("sv_emb", (1, 20480), "tensor(float)"))
    OUTPUTS = (NodeArg("ge", (1, 1024, 1), "tensor(float)"), NodeArg("ge_advanced", (1, 512, 1), "tensor(float)"))

    def run(self, output_names, input_feed):
        self._need(input_feed, "ref_audio", "sv_emb")
        ge, ga = self.engine.prompt_encode(input_feed["ref_audio"], input_feed["sv_emb"])
        return self._select(output_names, {"ge": _np(ge).reshape(1, 1024, 1),
                                           "ge_advanced": _np(ga).reshape(1, 512, 1)})


class HubertSession(_Session):
    """chinese-hubert-base.onnx, CN-HuBERT (reference call: ReferenceAudio.py:50-52):
    raw 16 kHz audio -> ssl_content [1, 768, T]."""
    INPUTS = (NodeArg("input_values", (1, "N"), "tensor(float)"),)
    OUTPUTS = (NodeArg("ssl_content", (1, 768, "T"), "tensor(float)"),)

    def run(self, output_names, input_feed):
        self._need(input_feed, "input_values")
        ssl = self.engine.hubert(input_feed["input_values"])
        return self._select(output_names, {"ssl_content": _np(ssl)[None]})


class SvSession(_Session):
    """speaker_encoder.onnx, V2ProPlus speaker verification (reference call:
    ReferenceAudio.py:71-72): waveform = 16 kHz clip [1, N] -> sv_emb [1, 20480]."""
    INPUTS = (NodeArg("waveform", (1, "N"), "tensor(float)"),)
    OUTPUTS = (NodeArg("sv_emb", (1, 20480), "tensor(float)"),)

    def run(self, output_names, input_feed):
        self._need(input_feed, "waveform")
        return self._select(output_names, {"sv_emb": _np(self.engine.sv(input_feed["waveform"]))})


class RobertaSession(_Session):
    """RoBERTa.onnx, Chinese BERT features (reference call: GetPhonesAndBert.py:64-74):
    input_ids [1, N], attention_mask [1, N], repeats = word2ph [n_chars] ->
    text_bert [sum(repeats), 1024]."""
    INPUTS = (NodeArg("input_ids", (1, "N"), "tensor(int64)"), NodeArg("attention_mask", (1, "N"), "tensor(int64)"),
              NodeArg("repeats", ("C",), "tensor(int64)"))
    OUTPUTS = (NodeArg("text_bert", ("P", 1024), "tensor(float)"),)

    def run(self, output_names, input_feed):
        self._need(input_feed, "input_ids", "attention_mask", "repeats")
        f = input_feed
        out = self.engine.roberta(f["input_ids"], f["repeats"], f["attention_mask"])
        return self._select(output_names, {"text_bert": _np(out)})
