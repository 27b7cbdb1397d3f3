"""Read the initializer table (name, dims, external offset/length) of a Genie graph.

The character directory's relinked graphs carry the tensor layout of the
fp16/fp32 weight bins as ONNX external-data entries (`g/ModelManager.py:80-103`).
Only the fields that table needs are decoded from the protobuf wire format
(ModelProto.graph=7; GraphProto.initializer=5; TensorProto dims=1, name=8,
external_data=13{key=1,value=2}, data_location=14).  The `onnx` package is
not a dependency of this engine.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple


def _varint(b: bytes, p: int) -> Tuple[int, int]:
    r = s = 0
    while True:
        c = b[p]
        p += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, p
        s += 7


def _walk(b: bytes):
    p, n = 0, len(b)
    while p < n:
        k, p = _varint(b, p)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, p = _varint(b, p)
        elif wt == 2:
            ln, p = _varint(b, p)
            v = b[p:p + ln]
            p += ln
        elif wt == 1:
            v, p = b[p:p + 8], p + 8
        elif wt == 5:
            v, p = b[p:p + 4], p + 4
        else:
            raise ValueError(f"bad wire type {wt}")
        yield f, wt, v


def _tensor_entry(b: bytes):
    name = ""
    dims: List[int] = []
    ext: Dict[str, str] = {}
    for f, wt, v in _walk(b):
        if f == 1:
            if wt == 0:
                dims.append(v)
            else:
                q = 0
                while q < len(v):
                    d, q = _varint(v, q)
                    dims.append(d)
        elif f == 8:
            name = bytes(v).decode()
        elif f == 13:
            key = val = ""
            for f2, _, v2 in _walk(v):
                if f2 == 1:
                    key = bytes(v2).decode()
                elif f2 == 2:
                    val = bytes(v2).decode()
            ext[key] = val
    off: Optional[int] = int(ext["offset"]) if "offset" in ext else None
    ln: Optional[int] = int(ext["length"]) if "length" in ext else None
    return name, dims, off, ln


def read_initializer_table(path: str) -> Dict[str, Tuple[List[int], Optional[int], Optional[int]]]:
    with open(path, "rb") as fh:
        buf = fh.read()
    table = {}
    for f, _, v in _walk(buf):
        if f != 7:
            continue
        for f2, _, v2 in _walk(v):
            if f2 == 5:
                name, dims, off, ln = _tensor_entry(v2)
                table[name] = (dims, off, ln)
    return table


def read_initializer_values(path: str, spec) -> Dict[str, "object"]:
    """Inline initializers (TensorProto data_type=2 field, raw_data=9) of a graph
    whose weights are stored in the file itself (RoBERTa.onnx is loaded without an
    fp16 bin, `g/ModelManager.py:139`): FLOAT (1) or FLOAT16 (10) raw data, checked
    against `spec` (name -> shape)."""
    import numpy as np
    with open(path, "rb") as fh:
        buf = fh.read()
    found = {}
    for f, _, v in _walk(buf):
        if f != 7:
            continue
        for f2, _, v2 in _walk(v):
            if f2 != 5:
                continue
            name, dims, dtype, raw = "", [], 0, b""
            for f3, wt, v3 in _walk(v2):
                if f3 == 1:
                    if wt == 0:
                        dims.append(v3)
                    else:
                        q = 0
                        while q < len(v3):
                            d, q = _varint(v3, q)
                            dims.append(d)
                elif f3 == 2:
                    dtype = v3
                elif f3 == 8:
                    name = bytes(v3).decode()
                elif f3 == 9:
                    raw = bytes(v3)
            if name in spec:
                dt = {1: np.float32, 10: np.float16}.get(dtype)
                if dt is None or not raw:
                    raise ValueError(f"{path}: {name} has no inline FLOAT/FLOAT16 raw data")
                found[name] = np.frombuffer(raw, dtype=dt).reshape(dims)
    out = {}
    for name, shape in spec.items():
        if name not in found:
            raise KeyError(f"{path}: initializer {name} not found")
        if tuple(found[name].shape) != tuple(shape):
            raise ValueError(f"{name}: shape {found[name].shape} in graph, expected {shape}")
        out[name] = found[name]
    return out


def _inline_array(v2):
    """(name, ndarray or None) of an inline TensorProto (FLOAT / FLOAT16 raw_data)."""
    import numpy as np
    name, dims, dtype, raw = "", [], 0, b""
    for f3, wt, v3 in _walk(v2):
        if f3 == 1:
            if wt == 0:
                dims.append(v3)
            else:
                q = 0
                while q < len(v3):
                    d, q = _varint(v3, q)
                    dims.append(d)
        elif f3 == 2:
            dtype = v3
        elif f3 == 8:
            name = bytes(v3).decode()
        elif f3 == 9:
            raw = bytes(v3)
    dt = {1: np.float32, 10: np.float16}.get(dtype)
    arr = np.frombuffer(raw, dtype=dt).reshape(dims) if dt is not None and raw else None
    return name, arr


def read_graph(path: str):
    """Inline initializers and nodes of a graph: ({name: ndarray}, [(op_type, inputs,
    outputs, node name)] in file order, which torch.onnx.export writes topologically).
    NodeProto: input=1, output=2, name=3, op_type=4; GraphProto: node=1, initializer=5."""
    with open(path, "rb") as fh:
        buf = fh.read()
    inits, nodes = {}, []
    for f, _, v in _walk(buf):
        if f != 7:
            continue
        for f2, _, v2 in _walk(v):
            if f2 == 5:
                name, arr = _inline_array(v2)
                if arr is not None:
                    inits[name] = arr
            elif f2 == 1:
                ins, outs, nm, op = [], [], "", ""
                for f3, _, v3 in _walk(v2):
                    if f3 == 1:
                        ins.append(bytes(v3).decode())
                    elif f3 == 2:
                        outs.append(bytes(v3).decode())
                    elif f3 == 3:
                        nm = bytes(v3).decode()
                    elif f3 == 4:
                        op = bytes(v3).decode()
                nodes.append((op, ins, outs, nm))
    return inits, nodes
