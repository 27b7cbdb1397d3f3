"""Minimal protobuf wire-format reader for ONNX ModelProto (oracle tooling).

TEST INFRASTRUCTURE ONLY. Used in this container to read the reference graph
templates `src/genie_tts/Data/{v2,v2ProPlus}/Models/*.onnx` (which the reference
loads with `onnx.load(..., load_external_data=False)`, `g/ModelManager.py:74`)
without the `onnx` package, which is absent here.  Field numbers follow the
public onnx.proto (ModelProto.graph=7, GraphProto.node=1, initializer=5,
input=11, output=12; NodeProto.input=1, output=2, name=3, op_type=4,
attribute=5; AttributeProto name=1 f=2 i=3 s=4 t=5 g=6 floats=7 ints=8
type=20; TensorProto dims=1 data_type=2 float_data=4 int32_data=5
int64_data=7 name=8 raw_data=9 double_data=10 external_data=13
data_location=14).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

# ONNX TensorProto.DataType -> numpy
ONNX_DTYPE = {
    1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32,
    7: np.int64, 9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32,
    13: np.uint64,
}


def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _fields(buf: bytes):
    """Yield (field_number, wire_type, value) for one message buffer."""
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, v


def _packed_varints(v, wt) -> List[int]:
    if wt == 0:
        return [v]
    out = []
    pos = 0
    while pos < len(v):
        x, pos = _varint(v, pos)
        out.append(x)
    return out


def _s64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


@dataclass
class Tensor:
    name: str = ""
    dims: List[int] = field(default_factory=list)
    data_type: int = 0
    raw: Optional[bytes] = None
    float_data: List[float] = field(default_factory=list)
    int64_data: List[int] = field(default_factory=list)
    int32_data: List[int] = field(default_factory=list)
    double_data: List[float] = field(default_factory=list)
    external: Dict[str, str] = field(default_factory=dict)
    data_location: int = 0

    @property
    def is_external(self) -> bool:
        return self.data_location == 1

    def numpy(self) -> np.ndarray:
        dt = ONNX_DTYPE[self.data_type]
        shape = tuple(self.dims)
        if self.raw is not None:
            return np.frombuffer(self.raw, dtype=dt).reshape(shape).copy()
        if self.float_data:
            return np.asarray(self.float_data, dtype=dt).reshape(shape)
        if self.int64_data:
            return np.asarray(self.int64_data, dtype=dt).reshape(shape)
        if self.int32_data:
            return np.asarray(self.int32_data, dtype=np.int32).astype(dt).reshape(shape)
        if self.double_data:
            return np.asarray(self.double_data, dtype=dt).reshape(shape)
        return np.zeros(shape, dtype=dt)


def parse_tensor(buf: bytes) -> Tensor:
    t = Tensor()
    for fno, wt, v in _fields(buf):
        if fno == 1:
            t.dims.extend(_s64(x) for x in _packed_varints(v, wt))
        elif fno == 2:
            t.data_type = v
        elif fno == 4:
            if wt == 2:
                t.float_data.extend(struct.unpack(f"<{len(v)//4}f", v))
            else:
                t.float_data.append(struct.unpack("<f", v)[0])
        elif fno == 5:
            t.int32_data.extend(_s64(x) for x in _packed_varints(v, wt))
        elif fno == 7:
            t.int64_data.extend(_s64(x) for x in _packed_varints(v, wt))
        elif fno == 8:
            t.name = v.decode()
        elif fno == 9:
            t.raw = bytes(v)
        elif fno == 10:
            if wt == 2:
                t.double_data.extend(struct.unpack(f"<{len(v)//8}d", v))
            else:
                t.double_data.append(struct.unpack("<d", v)[0])
        elif fno == 13:
            k = val = None
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    k = v2.decode()
                elif f2 == 2:
                    val = v2.decode()
            t.external[k] = val
        elif fno == 14:
            t.data_location = v
    return t


@dataclass
class Node:
    op_type: str
    name: str
    inputs: List[str]
    outputs: List[str]
    attrs: Dict[str, Any]


@dataclass
class Graph:
    name: str
    nodes: List[Node]
    initializers: Dict[str, Tensor]
    init_order: List[str]
    inputs: List[Tuple[str, int, List[Any]]]
    outputs: List[Tuple[str, int, List[Any]]]


def parse_attr(buf: bytes) -> Tuple[str, Any]:
    name = None
    val: Any = None
    floats: List[float] = []
    ints: List[int] = []
    atype = 0
    for fno, wt, v in _fields(buf):
        if fno == 1:
            name = v.decode()
        elif fno == 2:
            val = struct.unpack("<f", v)[0]
        elif fno == 3:
            val = _s64(v)
        elif fno == 4:
            val = bytes(v)
        elif fno == 5:
            val = parse_tensor(v)
        elif fno == 6:
            val = parse_graph(v)
        elif fno == 7:
            if wt == 2:
                floats.extend(struct.unpack(f"<{len(v)//4}f", v))
            else:
                floats.append(struct.unpack("<f", v)[0])
        elif fno == 8:
            ints.extend(_s64(x) for x in _packed_varints(v, wt))
        elif fno == 20:
            atype = v
    if atype == 6 or (val is None and floats):
        val = floats
    elif atype == 7 or (val is None and ints):
        val = ints
    return name, val


def parse_value_info(buf: bytes):
    name = ""
    elem = 0
    dims: List[Any] = []
    for fno, _, v in _fields(buf):
        if fno == 1:
            name = v.decode()
        elif fno == 2:
            for f2, _, v2 in _fields(v):
                if f2 == 1:  # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 1:
                            elem = v3
                        elif f3 == 2:
                            for f4, _, v4 in _fields(v3):
                                if f4 == 1:
                                    d: Any = None
                                    for f5, _, v5 in _fields(v4):
                                        if f5 == 1:
                                            d = _s64(v5)
                                        elif f5 == 2:
                                            d = v5.decode()
                                    dims.append(d)
    return name, elem, dims


def parse_node(buf: bytes) -> Node:
    ins: List[str] = []
    outs: List[str] = []
    name = ""
    op = ""
    attrs: Dict[str, Any] = {}
    for fno, _, v in _fields(buf):
        if fno == 1:
            ins.append(v.decode())
        elif fno == 2:
            outs.append(v.decode())
        elif fno == 3:
            name = v.decode()
        elif fno == 4:
            op = v.decode()
        elif fno == 5:
            k, val = parse_attr(v)
            attrs[k] = val
    return Node(op, name, ins, outs, attrs)


def parse_graph(buf: bytes) -> Graph:
    nodes: List[Node] = []
    inits: Dict[str, Tensor] = {}
    order: List[str] = []
    inputs = []
    outputs = []
    name = ""
    for fno, _, v in _fields(buf):
        if fno == 1:
            nodes.append(parse_node(v))
        elif fno == 2:
            name = v.decode()
        elif fno == 5:
            t = parse_tensor(v)
            inits[t.name] = t
            order.append(t.name)
        elif fno == 11:
            inputs.append(parse_value_info(v))
        elif fno == 12:
            outputs.append(parse_value_info(v))
    init_names = set(inits)
    inputs = [i for i in inputs if i[0] not in init_names]
    return Graph(name, nodes, inits, order, inputs, outputs)


def load_model(path: str) -> Graph:
    with open(path, "rb") as f:
        buf = f.read()
    graph = None
    for fno, _, v in _fields(buf):
        if fno == 7:
            graph = parse_graph(v)
    if graph is None:
        raise ValueError(f"{path}: no graph")
    return graph
