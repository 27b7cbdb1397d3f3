"""Phase timeline of the persistent decode launch (step 8, layer 12), option ptrace.

Group 0 (owns layer 12).  attention workgroups (0..15): 0 before the x_l wait, 1 x_l
ready, 2 q/k/v ready, 3 softmax numerators ready, 4 head output ready, 5 partials
published, 6 h1 ready.  FFN workgroups (16..79): 0 before the x_l wait, 1 x_l ready,
2 head partials summed, 6 h1 ready, 3 FFN1 done, 4 FFN2 partials published,
5 reduce-F published.  Microseconds from the first stamp."""
import sys
sys.path.insert(0, ".")
import numpy as np
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler

w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
e.set_option("ptrace", 1)
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
e.set_timing(True)
for rep in range(3):
    e.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=81))
print("decode ms", e.timing()[2], "kernel us", e.kernel_timing())
tr = e.ptrace().astype(np.int64)
# owners of the probed layer: attention workgroups stamp q/k/v (slot 2) and the FFN owners FFN1 (slot 3)
per = 16 + 64   # B=1: 16 attention + 64 FFN workgroups per layer group
grp = [g for g in range(256 // per) if (tr[g * per:(g + 1) * per, :8] > 0).any()]
G = len(grp)
og = 12 % G
att, ffn = tr[og * per:og * per + 16, :8], tr[og * per + 16:(og + 1) * per, :8]
ck = tr[og * per:og * per + 16, 8:16]
print(f"groups {G}, owner group {og}")
print("shader clock MHz (attention, stamp 1->2):", np.median((ck[:, 2] - ck[:, 1]) / ((att[:, 2] - att[:, 1]) * 10e-3)))
t0 = att[:, 0].min()
for nm, t in (("attn", att), ("ffn", ffn)):
    t = (t - t0) * 10 / 1000.0
    print(f"{nm:5s} " + "  ".join(f"s{i} min {t[:, i].min():6.2f} med {np.median(t[:, i]):6.2f} max {t[:, i].max():6.2f}"
                               for i in range(8) if -1e5 < t[:, i].max() < 1e5))
