"""Sampler ablation timings (in-graph average per launch)."""
import sys
sys.path.insert(0, ".")
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler
w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
e.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=40))
names = {0: "empty1", 14: "sample", 15: "no_topk", 16: "no_softmax", 17: "loads_tail"}
print(" ".join(f"{n}={e.probe(i, 1, 400):.2f}us" for i, n in names.items()), flush=True)
