"""Per-wave view of one layer of the single-sequence persistent decode: run with
GENIE_ENGINE_LIB pointing at a build whose ptrace slots 8..15 hold each wave's stamp
before the FFN1 barrier (FFN workgroups) / after its attention share (attention
workgroups) -- tools/build_alt.sh with a stamped variant.  Microseconds from the
first layer-12 attention stamp; slot meanings as tools/ptrace2.py."""
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
    t = (tr[b:b + 16] - t0) * 10 / 1000.0
    print(f"{nm:6s} " + "  ".join(f"s{i} {np.median(t[:, i]):6.2f}" for i in range(8) if -1e5 < t[:, i].max() < 1e5))
    for blk in (0, 5):
        print(f"   block {b + blk} slots 8..15: " + " ".join(f"{x:6.2f}" for x in t[blk, 8:16]))
