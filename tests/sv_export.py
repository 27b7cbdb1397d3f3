"""Test helper: write synthetic SV weights (weights.sv_spec, state-dict layout) as the
kind of speaker_encoder.onnx an exporter produces when it renames initializers
(onnx::Conv_N): Conv nodes in forward3's execution order (weights.sv_conv_order),
either followed by BatchNormalization nodes or with BatchNorm folded into the convs
(w g / sqrt(var + eps), (b - mean) g / sqrt(var + eps) + beta, in float32 as the
engine folds it).  Only the graph structure the loader reads is written."""
from __future__ import annotations

import numpy as np

from genie_tts_amd import weights as W
from tests.onnx_writer import model_graph

EPS = np.float32(1e-5)


def fold(w, conv, bn):
    wt = np.asarray(w[conv + ".weight"], np.float32)
    b = np.asarray(w.get(conv + ".bias", np.zeros(wt.shape[0], np.float32)), np.float32)
    if bn is None:
        return wt, (b if conv + ".bias" in w else None)
    s = (w[bn + ".weight"] / np.sqrt(w[bn + ".running_var"] + EPS)).astype(np.float32)
    return (wt * s[:, None, None, None]).astype(np.float32), ((b - w[bn + ".running_mean"]) * s + w[bn + ".bias"]).astype(np.float32)


def export(w, path, folded: bool):
    arrays, nodes, k = {}, [], 0
    x = "input"
    for conv, bn in W.sv_conv_order():
        scope = "/" + conv.replace(".", "/")
        if folded:
            wt, b = fold(w, conv, bn)
        else:
            wt, b = np.asarray(w[conv + ".weight"], np.float32), w.get(conv + ".bias")
        wn, bn_name = f"onnx::Conv_{k}", f"onnx::Conv_{k + 1}"
        k += 2
        arrays[wn] = wt
        ins = [x, wn]
        if b is not None:
            arrays[bn_name] = np.asarray(b, np.float32)
            ins.append(bn_name)
        y = f"{scope}/Conv_output_0"
        nodes.append(("Conv", ins, [y], f"{scope}/Conv"))
        if bn is not None and not folded:
            names = []
            for leaf in ("weight", "bias", "running_mean", "running_var"):
                names.append(f"onnx::BN_{k}")
                arrays[names[-1]] = np.asarray(w[f"{bn}.{leaf}"], np.float32)
                k += 1
            z = f"{scope}/BN_output_0"
            nodes.append(("BatchNormalization", [y] + names, [z], f"{scope}/BatchNormalization"))
            y = z
        x = y
    with open(path, "wb") as f:
        f.write(model_graph(arrays, nodes))
