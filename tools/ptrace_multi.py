"""Per-sequence timeline of the multi-sequence persistent decode (k_decode_persist1m): B = 8
copies of the bench utterance, step 8; for each layer group's attention / FFN workgroups
(first owned layer = the group index) the start and end of sequences 0..3's passes, then
the phase stamps of sequence 1's pass (attention: stage checked, x formed, q/k/v + K/V
landed, attention merged, before / after publishing; FFN: x formed, head partials summed,
FFN1 done, before / after publishing, end, LN1 input formed, FFN1 MFMA done), in us from
the first stamp.
Usage: python tools/ptrace_multi.py [B]"""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from genie_tts_amd import synth, workloads
from genie_tts_amd.engine import Engine, make_sampler

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
wl = workloads.single()
ref, it = wl.reference, wl.items[0]
e = Engine(synth.synthetic_character("v2"), "v2")
e.set_option("persist", 1)
e.set_option("ptrace", 1)
T = lambda a: torch.as_tensor(a, device="cuda")
utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)), it.force_steps)
for _ in range(3):
    e.t2s_generate([utt] * B, make_sampler())
tr = e.ptrace().astype(np.int64)
G = tr.shape[0] // 32
nz = tr[tr > 0]
t0 = nz.min()
us = lambda x: (x - t0) * 10 / 1000.0
for g in range(G):
    for role, off in (("attn", 0), ("ffn", 16)):
        rows = tr[32 * g + off: 32 * g + off + 16]
        st = [us(np.median(rows[:, 2 * b])) for b in range(min(B, 4))]
        en = [us(np.median(rows[:, 2 * b + 1])) for b in range(min(B, 4))]
        ph = [us(np.median(rows[:, 8 + k])) for k in range(8 if role == "ffn" else 6)]
        print(f"group {g} {role:4s} " + " ".join(f"[{a:7.2f} {z:7.2f}]" for a, z in zip(st, en))
              + "  seq1: " + " ".join(f"{p:7.2f}" for p in ph))
