"""Microbenchmark the decode-step kernels (in-graph average time per launch)."""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler
w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
for B in (1,):
    e.t2s_generate([(ref, txt, None, None, ssl)] * B, make_sampler(force_steps=40))
    names = ["empty1", "empty256", "qkv+ln", "qkv", "ffn1+ln", "ffn2", "outproj", "attn", "step", "attn_out", "ffn_fused", "qkv_part"]
    res = {n: e.probe(i, B, 400 if i != 8 else 50) for i, n in enumerate(names)}
    print(f"B={B} " + " ".join(f"{k}={v:.2f}us" for k, v in res.items()), flush=True)
