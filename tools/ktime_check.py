"""Diagnostic: does the in-graph event pair around the probed decode kernel time?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler
w = synth.synthetic_character("v2")
eng = Engine(w, "v2", device=0)
ref = synth.synth_phones(48, "a"); txt = synth.synth_phones(45, "b"); ssl = synth.synth_ssl(264, "c")
eng.set_timing(True)
for i in range(3):
    eng.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=81))
    print("kernel_timing", eng.kernel_timing(), flush=True)
