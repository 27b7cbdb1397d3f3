"""Numpy executor for the reference ONNX graph templates (oracle tooling).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Executes the six graphs
shipped in the reference (`src/genie_tts/Data/{v2,v2ProPlus}/Models/*.onnx`)
node by node, following the public ONNX operator semantics (opset 20), the
same graphs the reference runs through `onnxruntime.InferenceSession.run`
(`g/Core/Inference.py:47,55,76,88,102`).  Weights are supplied by the caller
(the reference patches them into the graph from the fp16 bin,
`g/ModelManager.py:59-114`).

`RandomNormalLike` is the only non-deterministic op in the graphs
(`t2s_stage_decoder_fp32.onnx#1799`, `t2s_first_stage_decoder_fp32.onnx#1813`,
`vits_fp32.onnx(v2)#6490`, `(v2pp)#6225`); callers substitute it with a
deterministic tensor through `random_normal` (a callable taking the input and
returning the sample), e.g. ones for the T2S greedy definition and zeros /
a committed epsilon for VITS.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np

from .onnx_wire import Graph, Node, ONNX_DTYPE, Tensor


def _np_dtype(code: int):
    return ONNX_DTYPE[code]


def _conv1d(x, w, b, stride, pad, dil, group):
    # x [N, C, L], w [O, C/g, K]
    n, c, l = x.shape
    o, cg, k = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad[0], pad[1])))
    lout = (xp.shape[2] - dil * (k - 1) - 1) // stride + 1
    out = np.zeros((n, o, lout), dtype=np.float32)
    og = o // group
    for g in range(group):
        xg = xp[:, g * cg:(g + 1) * cg, :]
        wg = w[g * og:(g + 1) * og]
        # im2col: [N, cg*k, lout]
        cols = np.empty((n, cg, k, lout), dtype=np.float32)
        for kk in range(k):
            st = kk * dil
            cols[:, :, kk, :] = xg[:, :, st: st + stride * (lout - 1) + 1: stride]
        out[:, g * og:(g + 1) * og, :] = np.einsum(
            "ok,nkl->nol", wg.reshape(og, cg * k), cols.reshape(n, cg * k, lout),
            optimize=True)
    if b is not None:
        out += b.reshape(1, -1, 1)
    return out


def _conv(x, w, b, attrs):
    nd = w.ndim - 2
    stride = attrs.get("strides", [1] * nd)
    dil = attrs.get("dilations", [1] * nd)
    pads = attrs.get("pads", [0] * (2 * nd))
    group = attrs.get("group", 1)
    if attrs.get("auto_pad", b"NOTSET") not in (b"NOTSET", "NOTSET"):
        raise NotImplementedError("auto_pad")
    if nd == 1:
        return _conv1d(x, w, b, stride[0], (pads[0], pads[1]), dil[0], group)
    if nd == 2:
        # only used as (k, 1) kernels?  generic via folding second dim
        raise NotImplementedError("2-D conv")
    raise NotImplementedError(f"{nd}-D conv")


def _conv_transpose1d(x, w, b, attrs):
    # x [N, Cin, L], w [Cin, Cout/g, K]
    stride = attrs.get("strides", [1])[0]
    dil = attrs.get("dilations", [1])[0]
    pads = attrs.get("pads", [0, 0])
    group = attrs.get("group", 1)
    outpad = attrs.get("output_padding", [0])[0]
    if group != 1:
        raise NotImplementedError("grouped ConvTranspose")
    n, cin, l = x.shape
    _, cout, k = w.shape
    full = (l - 1) * stride + dil * (k - 1) + 1 + outpad
    out = np.zeros((n, cout, full), dtype=np.float32)
    for kk in range(k):
        contrib = np.einsum("co,ncl->nol", w[:, :, kk], x, optimize=True)
        st = kk * dil
        out[:, :, st: st + stride * (l - 1) + 1: stride] += contrib
    out = out[:, :, pads[0]: full - pads[1]]
    if b is not None:
        out = out + b.reshape(1, -1, 1)
    return out.astype(np.float32)


def _stft(signal, frame_step, window, frame_length, onesided):
    # signal [B, L, 1] real
    sig = signal[..., 0] if signal.ndim == 3 else signal
    fl = int(frame_length) if frame_length is not None else window.shape[0]
    step = int(frame_step)
    bsz, length = sig.shape
    nfr = 1 + (length - fl) // step
    frames = np.stack([sig[:, i * step: i * step + fl] for i in range(nfr)], axis=1)
    if window is not None:
        frames = frames * window.reshape(1, 1, -1)
    spec = np.fft.rfft(frames.astype(np.float64), axis=-1) if onesided else \
        np.fft.fft(frames.astype(np.float64), axis=-1)
    out = np.stack([spec.real, spec.imag], axis=-1).astype(np.float32)
    return out


class Interpreter:
    def __init__(self, graph: Graph, weights: Dict[str, np.ndarray],
                 random_normal: Optional[Callable[[np.ndarray, dict], np.ndarray]] = None,
                 trace: Optional[Callable[[int, Node, List[np.ndarray]], None]] = None):
        self.graph = graph
        self.weights = weights
        self.random_normal = random_normal
        self.trace = trace

    def run(self, feeds: Dict[str, np.ndarray], fetch: Optional[List[str]] = None):
        env: Dict[str, np.ndarray] = {}
        for name, t in self.graph.initializers.items():
            if name in self.weights:
                env[name] = np.asarray(self.weights[name])
            elif not t.is_external:
                env[name] = t.numpy()
            else:
                raise KeyError(f"missing weight {name}")
        env.update({k: np.asarray(v) for k, v in feeds.items()})
        self._exec(self.graph, env, top=True)
        names = fetch or [o[0] for o in self.graph.outputs]
        return [env[n] for n in names]

    def _exec(self, graph: Graph, env: Dict[str, np.ndarray], top=False):
        for idx, node in enumerate(graph.nodes):
            ins = [env[i] if i else None for i in node.inputs]
            outs = self._op(node, ins, env)
            if not isinstance(outs, (list, tuple)):
                outs = [outs]
            for name, val in zip(node.outputs, outs):
                if name:
                    env[name] = val
            if top and self.trace is not None:
                self.trace(idx, node, outs)

    # ------------------------------------------------------------------ ops
    def _op(self, node: Node, ins, env):
        op = node.op_type
        a = node.attrs
        f = getattr(self, "op_" + op, None)
        if f is None:
            raise NotImplementedError(op)
        return f(ins, a, env, node)

    def op_Constant(self, ins, a, env, node):
        if "value" in a:
            return a["value"].numpy()
        if "value_float" in a:
            return np.array(a["value_float"], dtype=np.float32)
        if "value_int" in a:
            return np.array(a["value_int"], dtype=np.int64)
        if "value_ints" in a:
            return np.array(a["value_ints"], dtype=np.int64)
        if "value_floats" in a:
            return np.array(a["value_floats"], dtype=np.float32)
        raise NotImplementedError(str(a.keys()))

    def op_ConstantOfShape(self, ins, a, env, node):
        val = a["value"].numpy().reshape(-1)[0] if "value" in a else np.float32(0)
        return np.full(tuple(int(x) for x in ins[0]), val, dtype=np.asarray(val).dtype)

    def op_Shape(self, ins, a, env, node):
        shp = np.array(ins[0].shape, dtype=np.int64)
        st = a.get("start", 0)
        en = a.get("end", None)
        return shp[st:en]

    def op_Cast(self, ins, a, env, node):
        return ins[0].astype(_np_dtype(a["to"]))

    def _bin(self, ins, fn):
        x, y = ins
        r = fn(x, y)
        if x.dtype == np.float32 or y.dtype == np.float32:
            r = np.asarray(r)
            if r.dtype == np.float64:
                r = r.astype(np.float32)
        return r

    def op_Add(self, ins, a, env, node):
        return self._bin(ins, np.add)

    def op_Sub(self, ins, a, env, node):
        return self._bin(ins, np.subtract)

    def op_Mul(self, ins, a, env, node):
        return self._bin(ins, np.multiply)

    def op_Div(self, ins, a, env, node):
        x, y = ins
        if np.issubdtype(x.dtype, np.integer):
            q = np.floor_divide(np.abs(x), np.abs(y)) * np.sign(x) * np.sign(y)
            return q.astype(x.dtype)
        return self._bin(ins, np.divide)

    def op_Pow(self, ins, a, env, node):
        x, y = ins
        r = np.power(x, y.astype(x.dtype) if x.dtype.kind == "f" else y)
        return r.astype(x.dtype)

    def op_Max(self, ins, a, env, node):
        r = ins[0]
        for t in ins[1:]:
            r = np.maximum(r, t)
        return r

    def op_Equal(self, ins, a, env, node):
        return np.equal(ins[0], ins[1])

    def op_Greater(self, ins, a, env, node):
        return np.greater(ins[0], ins[1])

    def op_Less(self, ins, a, env, node):
        return np.less(ins[0], ins[1])

    def op_Or(self, ins, a, env, node):
        return np.logical_or(ins[0], ins[1])

    def op_Not(self, ins, a, env, node):
        return np.logical_not(ins[0])

    def op_Neg(self, ins, a, env, node):
        return np.negative(ins[0])

    def op_Sqrt(self, ins, a, env, node):
        return np.sqrt(ins[0])

    def op_Exp(self, ins, a, env, node):
        return np.exp(ins[0])

    def op_Sin(self, ins, a, env, node):
        return np.sin(ins[0])

    def op_Cos(self, ins, a, env, node):
        return np.cos(ins[0])

    def op_Tanh(self, ins, a, env, node):
        return np.tanh(ins[0])

    def op_Sigmoid(self, ins, a, env, node):
        x = ins[0]
        return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(x.dtype)

    def op_Softplus(self, ins, a, env, node):
        x = ins[0].astype(np.float64)
        return np.logaddexp(0.0, x).astype(ins[0].dtype)

    def op_Relu(self, ins, a, env, node):
        return np.maximum(ins[0], 0).astype(ins[0].dtype)

    def op_LeakyRelu(self, ins, a, env, node):
        x = ins[0]
        al = np.float32(a.get("alpha", 0.01))
        return np.where(x >= 0, x, x * al).astype(x.dtype)

    def op_PRelu(self, ins, a, env, node):
        x, s = ins
        return np.where(x >= 0, x, x * s).astype(x.dtype)

    def op_Where(self, ins, a, env, node):
        return np.where(ins[0], ins[1], ins[2])

    def op_Reshape(self, ins, a, env, node):
        x, shp = ins
        shp = [int(s) for s in shp]
        allowzero = a.get("allowzero", 0)
        out = []
        for i, s in enumerate(shp):
            if s == 0 and not allowzero:
                out.append(x.shape[i])
            else:
                out.append(s)
        return x.reshape(out)

    def op_Transpose(self, ins, a, env, node):
        perm = a.get("perm")
        return np.transpose(ins[0], perm)

    def op_Unsqueeze(self, ins, a, env, node):
        x = ins[0]
        axes = [int(v) for v in (ins[1] if len(ins) > 1 else a["axes"])]
        r = x.ndim + len(axes)
        axes = sorted(ax % r for ax in axes)
        for ax in axes:
            x = np.expand_dims(x, ax)
        return x

    def op_Squeeze(self, ins, a, env, node):
        x = ins[0]
        if len(ins) > 1 and ins[1] is not None:
            axes = tuple(int(v) % x.ndim for v in ins[1])
            return np.squeeze(x, axis=axes)
        return np.squeeze(x)

    def op_Concat(self, ins, a, env, node):
        return np.concatenate([i for i in ins], axis=a["axis"])

    def op_Split(self, ins, a, env, node):
        x = ins[0]
        axis = a.get("axis", 0)
        if len(ins) > 1 and ins[1] is not None:
            sizes = [int(s) for s in ins[1]]
        elif "split" in a:
            sizes = a["split"]
        else:
            n = len(node.outputs)
            tot = x.shape[axis]
            each = -(-tot // n)
            sizes = [min(each, tot - i * each) for i in range(n)]
        idx = np.cumsum(sizes)[:-1]
        return np.split(x, idx, axis=axis)

    def op_Slice(self, ins, a, env, node):
        x = ins[0]
        starts = [int(v) for v in ins[1]]
        ends = [int(v) for v in ins[2]]
        axes = [int(v) for v in ins[3]] if len(ins) > 3 and ins[3] is not None else list(range(len(starts)))
        steps = [int(v) for v in ins[4]] if len(ins) > 4 and ins[4] is not None else [1] * len(starts)
        sl = [slice(None)] * x.ndim
        for st, en, ax, sp in zip(starts, ends, axes, steps):
            ax %= x.ndim
            dim = x.shape[ax]
            if sp > 0:
                st = max(0, min(dim, st + dim if st < 0 else st))
                en = max(0, min(dim, en + dim if en < 0 else en))
            else:
                st = max(-1, min(dim - 1, st + dim if st < 0 else st))
                en = max(-1, min(dim - 1, en + dim if en < 0 else en))
                if en == -1:
                    en = None
            sl[ax] = slice(st, en, sp)
        return x[tuple(sl)]

    def op_Gather(self, ins, a, env, node):
        x, idx = ins
        axis = a.get("axis", 0)
        idx = np.where(idx < 0, idx + x.shape[axis], idx)
        return np.take(x, idx, axis=axis)

    def op_GatherElements(self, ins, a, env, node):
        x, idx = ins
        axis = a.get("axis", 0)
        idx = np.where(idx < 0, idx + x.shape[axis], idx)
        return np.take_along_axis(x, idx, axis=axis)

    def op_ScatterElements(self, ins, a, env, node):
        x, idx, upd = ins
        axis = a.get("axis", 0)
        red = a.get("reduction", b"none")
        if red not in (b"none", "none"):
            raise NotImplementedError("ScatterElements reduction")
        out = x.copy()
        idx = np.where(idx < 0, idx + x.shape[axis], idx)
        # sequential semantics (later duplicates win), as ORT's CPU loop
        it = np.nditer(idx, flags=["multi_index"])
        for v in it:
            mi = list(it.multi_index)
            src = tuple(mi)
            mi[axis] = int(v)
            out[tuple(mi)] = upd[src]
        return out

    def op_Expand(self, ins, a, env, node):
        x, shp = ins
        shp = [int(s) for s in shp]
        target = np.broadcast_shapes(x.shape, tuple(shp))
        return np.broadcast_to(x, target).copy()

    def op_Tile(self, ins, a, env, node):
        return np.tile(ins[0], [int(r) for r in ins[1]])

    def op_Pad(self, ins, a, env, node):
        x = ins[0]
        pads = [int(p) for p in ins[1]]
        cval = ins[2] if len(ins) > 2 and ins[2] is not None else None
        axes = [int(v) for v in ins[3]] if len(ins) > 3 and ins[3] is not None else list(range(x.ndim))
        mode = a.get("mode", b"constant")
        mode = mode.decode() if isinstance(mode, bytes) else mode
        na = len(axes)
        pw = [(0, 0)] * x.ndim
        for i, ax in enumerate(axes):
            pw[ax % x.ndim] = (pads[i], pads[i + na])
        # negative pads = crop
        crop = [slice(None)] * x.ndim
        pw2 = []
        for ax, (lo, hi) in enumerate(pw):
            s0 = -lo if lo < 0 else 0
            s1 = x.shape[ax] + hi if hi < 0 else x.shape[ax]
            crop[ax] = slice(s0, s1)
            pw2.append((max(lo, 0), max(hi, 0)))
        x = x[tuple(crop)]
        if mode == "constant":
            cv = 0 if cval is None else np.asarray(cval).reshape(-1)[0] if np.asarray(cval).size else 0
            return np.pad(x, pw2, mode="constant", constant_values=cv)
        if mode == "reflect":
            return np.pad(x, pw2, mode="reflect")
        if mode == "edge":
            return np.pad(x, pw2, mode="edge")
        raise NotImplementedError(mode)

    def op_CumSum(self, ins, a, env, node):
        x, axis = ins
        if a.get("exclusive", 0) or a.get("reverse", 0):
            raise NotImplementedError("CumSum flags")
        return np.cumsum(x, axis=int(axis)).astype(x.dtype)

    def _reduce_axes(self, ins, a, x):
        if len(ins) > 1 and ins[1] is not None and ins[1].size:
            return tuple(int(v) % x.ndim for v in ins[1])
        if "axes" in a:
            return tuple(int(v) % x.ndim for v in a["axes"])
        if a.get("noop_with_empty_axes", 0):
            return None
        return tuple(range(x.ndim))

    def op_ReduceSum(self, ins, a, env, node):
        x = ins[0]
        axes = self._reduce_axes(ins, a, x)
        if axes is None:
            return x
        return np.sum(x, axis=axes, keepdims=bool(a.get("keepdims", 1))).astype(x.dtype)

    def op_ReduceL2(self, ins, a, env, node):
        x = ins[0]
        axes = self._reduce_axes(ins, a, x)
        r = np.sqrt(np.sum(x.astype(np.float64) ** 2, axis=axes, keepdims=bool(a.get("keepdims", 1))))
        return r.astype(x.dtype)

    def op_ArgMax(self, ins, a, env, node):
        x = ins[0]
        axis = a.get("axis", 0)
        if a.get("select_last_index", 0):
            flipped = np.flip(x, axis=axis)
            r = x.shape[axis] - 1 - np.argmax(flipped, axis=axis)
        else:
            r = np.argmax(x, axis=axis)
        if a.get("keepdims", 1):
            r = np.expand_dims(r, axis)
        return r.astype(np.int64)

    def op_TopK(self, ins, a, env, node):
        x, k = ins
        k = int(np.asarray(k).reshape(-1)[0])
        axis = a.get("axis", -1) % x.ndim
        largest = a.get("largest", 1)
        key = -x if largest else x
        order = np.argsort(key, axis=axis, kind="stable")
        idx = np.take(order, np.arange(k), axis=axis)
        vals = np.take_along_axis(x, idx, axis=axis)
        return [vals, idx.astype(np.int64)]

    def op_Softmax(self, ins, a, env, node):
        x = ins[0]
        axis = a.get("axis", -1)
        m = np.max(x, axis=axis, keepdims=True)
        e = np.exp(x - m)
        return (e / np.sum(e, axis=axis, keepdims=True)).astype(x.dtype)

    def op_MatMul(self, ins, a, env, node):
        return np.matmul(ins[0], ins[1]).astype(np.float32)

    def op_Gemm(self, ins, a, env, node):
        A, B = ins[0], ins[1]
        C = ins[2] if len(ins) > 2 else None
        if a.get("transA", 0):
            A = A.T
        if a.get("transB", 0):
            B = B.T
        r = np.float32(a.get("alpha", 1.0)) * (A @ B)
        if C is not None:
            r = r + np.float32(a.get("beta", 1.0)) * C
        return r.astype(np.float32)

    def op_LayerNormalization(self, ins, a, env, node):
        x, scale = ins[0], ins[1]
        bias = ins[2] if len(ins) > 2 else None
        axis = a.get("axis", -1) % x.ndim
        eps = np.float32(a.get("epsilon", 1e-5))
        axes = tuple(range(axis, x.ndim))
        mu = np.mean(x, axis=axes, keepdims=True)
        var = np.mean((x - mu) ** 2, axis=axes, keepdims=True)
        y = (x - mu) / np.sqrt(var + eps) * scale
        if bias is not None:
            y = y + bias
        return y.astype(x.dtype)

    def op_Conv(self, ins, a, env, node):
        x, w = ins[0], ins[1]
        b = ins[2] if len(ins) > 2 else None
        return _conv(x.astype(np.float32), w.astype(np.float32), b, a)

    def op_ConvTranspose(self, ins, a, env, node):
        x, w = ins[0], ins[1]
        b = ins[2] if len(ins) > 2 else None
        return _conv_transpose1d(x.astype(np.float32), w.astype(np.float32), b, a)

    def op_STFT(self, ins, a, env, node):
        signal, frame_step = ins[0], ins[1]
        window = ins[2] if len(ins) > 2 else None
        frame_length = ins[3] if len(ins) > 3 else None
        return _stft(signal, np.asarray(frame_step).reshape(-1)[0], window,
                     None if frame_length is None else np.asarray(frame_length).reshape(-1)[0],
                     a.get("onesided", 1))

    def op_RandomNormalLike(self, ins, a, env, node):
        if self.random_normal is None:
            raise RuntimeError("RandomNormalLike needs a substitution (random_normal=)")
        return np.asarray(self.random_normal(ins[0], a), dtype=np.float32)

    def op_If(self, ins, a, env, node):
        cond = bool(np.asarray(ins[0]).reshape(-1)[0])
        sub = a["then_branch"] if cond else a["else_branch"]
        local = dict(env)
        for name, t in sub.initializers.items():
            local[name] = t.numpy()
        self._exec(sub, local)
        return [local[o[0]] for o in sub.outputs]
