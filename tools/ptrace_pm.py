"""Phase timeline of the batched persistent decode (k_decode_persistm): B copies of the
bench utterance, step 8; per stamp the median over the workgroups (us from the step's
start), then layer 12's phase durations.  Stamps: 12 step start, 13 tokens resolved,
0..7 layer 12 (attention role start, gather done, q/k/v done, attention done, PA
published, FFN gather done, FFN1 done, PFH published), 14 layer 23 done, 15 step end.
Usage: python tools/ptrace_pm.py [B]"""
import json
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from genie_tts_amd import synth, workloads
from genie_tts_amd.engine import Engine, make_sampler

B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 64
wl = workloads.single()
ref, it = wl.reference, wl.items[0]
e = Engine(synth.synthetic_character("v2"), "v2")
e.set_option("persist", 1)
e.set_option("persistm", 1)
e.set_option("persistm_min_b", 2)
e.set_option("ptrace", 1)
ATT = "--attn" in sys.argv
FFN = "--ffn" in sys.argv
if ATT:
    e.set_option("knob1", 1)
if FFN:
    e.set_option("knob1", 2)
if "--serial" in sys.argv:   # the serial per-sequence attention loop (knob2 = 1) instead of the concurrent one
    e.set_option("knob2", 1)
T = lambda a: torch.as_tensor(a, device="cuda")
utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)), it.force_steps)
for _ in range(3):
    e.t2s_generate([utt] * B, make_sampler())
tr = e.ptrace().astype(np.int64)
n = min(16, B) * 16
tr = tr[:n]
t0 = np.median(tr[:, 12])
us = lambda k: float(np.median(tr[:, k]) - t0) * 10 / 1000.0
names = {12: "step start", 13: "tokens resolved", 0: "L12 attn start", 1: "L12 gather done", 2: "L12 qkv done",
         3: "L12 attention done", 4: "L12 PA published", 5: "L12 FFN gather done", 6: "L12 FFN1 done",
         7: "L12 PFH published", 14: "L23 done", 8: "logits gather done", 9: "logits done",
         10: "candidates published", 15: "step end"}
if ATT:
    names.update({8: "L12 seq0 attention start", 9: "L12 seq1 attention start", 10: "L12 seq2 attention start",
                  11: "L12 seq3 attention start"})
    del names[14]
if FFN:
    names.update({8: "L12 FFN1 MFMA done (thread 0)", 9: "L12 W2 loads issued", 10: "L12 F written"})
    del names[14]
out = {"B": B, "workgroups": n, "us": {names[k]: round(us(k), 2) for k in ((12, 13, 0, 1, 2, 8, 9, 10, 11, 3, 4, 5, 6, 7, 15) if ATT else (12, 13, 0, 1, 2, 3, 4, 5, 8, 9, 10, 6, 7, 15) if FFN else (12, 13, 0, 1, 2, 3, 4, 5, 6, 7, 14, 8, 9, 10, 15))}}
spread = {names[k]: round(float(np.max(tr[:, k]) - np.min(tr[:, k])) * 10 / 1000.0, 2) for k in (0, 7)}
out["spread_us"] = spread
print(json.dumps(out))
