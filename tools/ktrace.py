"""Phase breakdown of the three decode kernels of layer 12 (GENIE_KTRACE=1).

Stamps are 100 MHz realtime counters written by thread 0 of each block.
QKV GEMV: 0 start, 1 prologue (partials + LN stats), 2 xs ready, 3 dots done, 4 end.
attention: 0 start, 1 all passes done, 2 merged o, 3 end.  FFN: 0 start, 1 partials + LN stats,
2 FFN1 done, 3 end."""
import os
import sys
sys.path.insert(0, ".")
os.environ["GENIE_KTRACE"] = "1"
import numpy as np
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler
w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
for rep in range(3):
    e.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=81))
tr = e.ktrace().astype(np.int64)
names = [("qkv", 192, 5), ("attn", 16, 4), ("ffn", 64, 4)]
t0 = min(int(tr[k, :n, 0].min()) for k, (_, n, _) in enumerate(names))
for k, (nm, n, ns) in enumerate(names):
    t = (tr[k, :n, :ns] - t0) * 10 / 1000.0      # us since the QKV kernel's first block
    print(f"{nm:5s} start min/med/max {t[:, 0].min():6.2f} {np.median(t[:, 0]):6.2f} {t[:, 0].max():6.2f}  "
          + "  ".join(f"s{i} med {np.median(t[:, i]):6.2f}" for i in range(1, ns))
          + f"  end max {t[:, ns - 1].max():6.2f}")
