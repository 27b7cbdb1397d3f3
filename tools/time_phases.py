"""Decode timing with hot vs. VITS-evicted caches (phase timers)."""
import sys
sys.path.insert(0, ".")
import numpy as np, torch
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler
import bench
w = synth.synthetic_character("v2")
e = Engine(w, "v2")
ref, txt, rb, tb, ssl, audio = bench.build_inputs()
sp = make_sampler(force_steps=bench.FORCE_STEPS)
e.set_timing(True)
for rep in range(3):
    sem = e.t2s_generate([(ref, txt, None, None, ssl)], sp)[0]
    print("t2s only      ", ["%.2f" % x for x in e.timing()[:3]], flush=True)
for rep in range(3):
    sem = e.t2s_generate([(ref, txt, None, None, ssl)], sp)[0]
    t = e.timing()[:3]
    wav = e.vits_decode(txt, sem, ref_audio=audio); torch.cuda.synchronize()
    print("t2s after vits", ["%.2f" % x for x in t], "vits %.2f" % e.timing()[3], flush=True)
print("probe step B=1 %.1f us" % e.probe(8, 1, 50))
print("probe step (8-step graph) %.1f us" % e.probe(12, 1, 80))
print("host launch of 8-step graph %.1f us" % e.probe(13, 1, 10))
for i, n in [(9, "attn_out"), (10, "ffn"), (11, "qkv_part")]:
    print(n, "%.2f us" % e.probe(i, 1, 400))
