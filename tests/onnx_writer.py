"""Minimal ONNX ModelProto writer for tests: a graph whose initializers are
EXTERNAL tensors (name, dims, offset, length) -- the shape of the relinked
graphs Genie's converter writes into a character directory."""
from __future__ import annotations

from typing import List, Tuple


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(no: int, wt: int, payload: bytes) -> bytes:
    return _varint((no << 3) | wt) + (_varint(len(payload)) + payload if wt == 2 else payload)


def _str(no: int, s: str) -> bytes:
    return _field(no, 2, s.encode())


def tensor_external(name: str, dims: List[int], offset: int, length: int, location: str) -> bytes:
    body = _field(1, 2, b"".join(_varint(d) for d in dims))
    body += _field(2, 0, _varint(1))              # FLOAT
    body += _str(8, name)
    for k, v in (("location", location), ("offset", str(offset)), ("length", str(length))):
        body += _field(13, 2, _str(1, k) + _str(2, v))
    body += _field(14, 0, _varint(1))             # EXTERNAL
    return body


def model(inits: List[Tuple[str, List[int], int, int]], location: str) -> bytes:
    graph = _str(2, "g")
    for name, dims, off, ln in inits:
        graph += _field(5, 2, tensor_external(name, dims, off, ln, location))
    return _field(1, 0, _varint(9)) + _field(7, 2, graph)


def tensor_inline(name: str, arr) -> bytes:
    """An initializer with its data in the file (raw_data), FLOAT or FLOAT16."""
    import numpy as np
    a = np.ascontiguousarray(arr)
    body = _field(1, 2, b"".join(_varint(d) for d in a.shape))
    body += _field(2, 0, _varint(10 if a.dtype == np.float16 else 1))
    body += _str(8, name)
    body += _field(9, 2, a.astype(a.dtype.newbyteorder("<")).tobytes())
    return body


def model_inline(arrays) -> bytes:
    graph = _str(2, "g")
    for name, a in arrays.items():
        graph += _field(5, 2, tensor_inline(name, a))
    return _field(1, 0, _varint(9)) + _field(7, 2, graph)


def node(op: str, inputs, outputs, name: str = "") -> bytes:
    body = b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outputs)
    if name:
        body += _str(3, name)
    return body + _str(4, op)


def model_graph(arrays, nodes) -> bytes:
    """Inline initializers plus nodes [(op_type, inputs, outputs, name)] in order."""
    graph = b"".join(_field(1, 2, node(*n)) for n in nodes) + _str(2, "g")
    for name, a in arrays.items():
        graph += _field(5, 2, tensor_inline(name, a))
    return _field(1, 0, _varint(9)) + _field(7, 2, graph)
