"""Two-layer phase timeline of the single-sequence persistent decode (t2s_persist1.hip),
step 8, layers 12 (group 4: attention WGs 128..143, FFN 144..159) and 13 (group 5:
attention 160..175, FFN 176..191).  Microseconds from the first layer-12 attention stamp.
attention: 0 before the x_l wait, 1 x_l ready, 2 q/k/v ready, 3 softmax numerators,
4 head output, 5 partials published.  FFN: 0 start, 1 woke / x_l ready, 2 head partials
summed, 6 h1 ready, 3 FFN1 done, 4 FFN2 partials published."""
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
print("decode ms", e.timing()[2])
tr = e.ptrace().astype(np.int64)
t0 = tr[128:144, 0].min()
for nm, b in (("attn12", 128), ("ffn12", 144), ("attn13", 160), ("ffn13", 176)):
    t = (tr[b:b + 16, :8] - t0) * 10 / 1000.0
    print(f"{nm:6s} " + "  ".join(f"s{i} {t[:, i].min():6.2f}/{np.median(t[:, i]):6.2f}/{t[:, i].max():6.2f}"
                                for i in range(8) if -1e5 < t[:, i].max() < 1e5))
if "--wg" in sys.argv:   # per-workgroup stamps of the FFN groups (late-publisher hunt)
    for nm, b in (("ffn12", 144), ("ffn13", 176)):
        t = (tr[b:b + 16, :8] - t0) * 10 / 1000.0
        for j in range(16):
            print(f"{nm} wg{j:2d} " + " ".join(f"s{i} {t[j, i]:7.2f}" for i in (0, 1, 2, 6, 3, 4)))
