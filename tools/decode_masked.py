"""Decode time of the single-sequence kernel alone: every CU vs the CU-masked engine
stream of the overlapped vocoder (no vocoder or prefetch work beside it)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from genie_tts_amd import synth  # noqa: E402
from genie_tts_amd.engine import Engine, make_sampler  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
e.set_timing(True)
for K in (0, 64, 0, 64):
    e.set_vocoder_cus(K)
    ts = []
    for _ in range(6):
        e.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=81))
        ts.append(e.timing()[2])
    print(K, "decode ms median", round(float(np.median(ts[1:])), 3), flush=True)
