"""Phase timeline of the persistent decode launch (step 8, layer 12), option ptrace.

attention workgroups (0..15): 0 cF(l-1) seen, 1 x_l ready, 2 attention merged,
3 accA published, 4 h1 ready, 5 qkv ready, 6 attention loop done.  FFN workgroups (16..79): 0 cA(l) seen, 1 LN1 done,
2 FFN1 done, 3 accF published, 4 x_{l+1} ready.  Microseconds from the first stamp."""
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
att, ffn = tr[:16, :7], tr[16:80, :7]
t0 = min(att[att > 0].min(), ffn[ffn > 0].min())
for nm, t in (("attn", att), ("ffn", ffn)):
    t = (t - t0) * 10 / 1000.0
    print(f"{nm:5s} " + "  ".join(f"s{i} min {t[:, i].min():6.2f} med {np.median(t[:, i]):6.2f} max {t[:, i].max():6.2f}"
                               for i in range(7) if t[:, i].max() > -1e5))
