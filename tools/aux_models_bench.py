"""Measured time of the reference-side models on the engine (SURVEY §8 "next" rows):
CN-HuBERT on a 5.3 s reference clip (ReferenceAudio.py:48-52, once per reference) and the
24-layer Chinese RoBERTa on a 20-character sentence (GetPhonesAndBert.py:64-74, once per
sentence), synthetic weights of the real shapes.  Prints one JSON line; the FLOP counts
are the dense-matmul work of each model, priced at the 157.3 TF/s f32 MFMA peak and at the
ceiling of the precision each kernel runs at: the f16 MFMA (2.5 PF dense) / MFMAs per product
(CN-HuBERT fp16 weights x split activations: 2; RoBERTa fp32 weights as hi + lo planes x
split activations: 3; SV fp32 weights: 3).  RoBERTa runs with fp32-valued weights, as
RoBERTa.onnx ships them (ModelManager.py:139-142)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from genie_tts_amd import synth, weights as W  # noqa: E402
from genie_tts_amd.engine import Engine, lib  # noqa: E402

torch.cuda.set_device(0)
out = {}
# ---- CN-HuBERT: 5.3 s at 16 kHz
eh = Engine({"hubert": synth.synth_weights(W.hubert_spec())}, "v2")
audio = torch.as_tensor(synth.rng_for("hb").standard_normal(int(16000 * 5.3)).astype(np.float32) * 0.1, device="cuda")
T = lib().gsv_hubert_frames(audio.numel())
for _ in range(3):
    eh.hubert(audio)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    eh.hubert(audio)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / n * 1e3
# conv stack + 12 transformer layers (768, FFN 3072) + pos conv (768 x 48 x 128 per group x 16)
conv = 2 * (T * 2 * 512 * 512 * 3 + T * 4 * 512 * 512 * 3 + T * 8 * 512 * 512 * 3 * 2 + T * 16 * 512 * 512 * 2)
layers = 12 * 2 * T * (768 * 2304 + 768 * 768 + 2 * 768 * 3072) + 12 * 4 * T * T * 768
pos = 2 * T * 768 * 48 * 128
flops = conv + layers + pos + 2 * T * 512 * 768
out["cn_hubert"] = {"audio_s": 5.3, "frames": int(T), "ms": ms, "gflop": flops / 1e9,
                    "frac_f32_peak": flops / 157.3e12 / (ms * 1e-3),
                    "frac_split_f16_peak": flops / (2500e12 / 2) / (ms * 1e-3)}
eh.close()
# ---- RoBERTa, 24 layers (hidden_states[-3]: 22 run), 20 characters
er = Engine({"roberta": synth.synth_weights(W.roberta_spec(24), fp16=False)}, "v2")
r = synth.rng_for("rbb")
n_chars = 20
ids = np.concatenate([[101], r.integers(672, 8000, size=n_chars), [102]]).astype(np.int64)
w2p = r.integers(1, 4, size=n_chars).astype(np.int64)
for _ in range(3):
    er.roberta(ids, w2p)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    er.roberta(ids, w2p)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / n * 1e3
N = ids.size
flops = 22 * (2 * N * (1024 * 3072 + 1024 * 1024 + 2 * 1024 * 4096) + 4 * N * N * 1024)
wbytes = 22 * (1024 * 3072 + 1024 * 1024 + 2 * 1024 * 4096) * 4   # hi + lo fp16 planes = fp32 bytes
out["roberta"] = {"tokens": int(N), "layers_run": 22, "ms": ms, "gflop": flops / 1e9,
                  "weight_planes_mb": wbytes / 1e6,
                  "frac_hbm_weights": wbytes / 8e12 / (ms * 1e-3),
                  "frac_split_f16_peak": flops / (2500e12 / 3) / (ms * 1e-3),
                  "w16_split_tensors": er.counter("w16_split_tensors")}
er.close()
# ---- speaker verification (V2ProPlus sv_emb, ReferenceAudio.py:71-72): 5.3 s + 0.3 s silence at 16 kHz
es = Engine({"sv": synth.synth_sv_weights()}, "v2")
audio = torch.as_tensor(synth.rng_for("sv").standard_normal(89600).astype(np.float32) * 0.1, device="cuda")
for _ in range(3):
    es.sv(audio)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    es.sv(audio)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / n * 1e3
T = lib().gsv_sv_frames(audio.numel())


def down(x):
    return (x - 1) // 2 + 1


flops, P, cin = 0, 80 * T, 64
flops += 2 * P * 64 * 9
F_, T_ = 80, T
for planes, nb, stride, aff in W.SV_STAGES:
    w = planes * 24 // 64
    for b in range(nb):
        s_ = stride if b == 0 else 1
        if s_ == 2:
            F_, T_ = down(F_), down(T_)
        P = F_ * T_
        flops += 2 * P * (cin * 4 * w + 4 * w * w * 9 + 4 * w * planes * 4)
        if b == 0 and (s_ != 1 or cin != planes * 4):
            flops += 2 * P * cin * planes * 4
        if aff:
            flops += 3 * 2 * P * (2 * w * (w // 4) + (w // 4) * w)
        cin = planes * 4
flops += 2 * P * 1024 * 9 * 2048 + 2 * P * (4096 * 512 + 512 * 2048)
out["sv"] = {"audio_s": 5.6, "frames": int(T), "ms": ms, "gflop": flops / 1e9,
             "frac_f32_peak": flops / 157.3e12 / (ms * 1e-3),
             "frac_split_f16_peak": flops / (2500e12 / 3) / (ms * 1e-3)}
es.close()
print(json.dumps(out), flush=True)
