"""Speaker-verification timing (gsv_sv) on a 5.3 s clip + 0.3 s silence, synthetic fp32
weights of the real shapes; run under rocprofv3 --kernel-trace --stats for the per-conv
breakdown.  Prints ms per call.  Usage: python tools/sv_bench.py [n_calls]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from genie_tts_amd import synth  # noqa: E402
from genie_tts_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.cuda.set_device(0)
e = Engine({"sv": synth.synth_sv_weights()}, "v2")
audio = torch.as_tensor(synth.rng_for("sv").standard_normal(89600).astype(np.float32) * 0.1, device="cuda")
for _ in range(3):
    e.sv(audio)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    e.sv(audio)
torch.cuda.synchronize()
print(f"sv {(time.perf_counter() - t0) / n * 1e3:.3f} ms per call", flush=True)
