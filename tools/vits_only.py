"""Run the bench's VITS phase alone (configs[1]: G=80, S=45, 5.3 s reference) N times
on cuda:0 -- a target for rocprofv3 kernel traces of the vocoder."""
import sys
import time
sys.path.insert(0, ".")
import numpy as np
import torch
from genie_tts_amd import synth, workloads
from genie_tts_amd.engine import Engine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
version = sys.argv[2] if len(sys.argv) > 2 else "v2"
w = synth.synthetic_character(version)
e = Engine(w, version)
wl = workloads.single()
txt = torch.as_tensor(wl.items[0].text_seq.reshape(-1), device="cuda")
sem = torch.as_tensor(synth.rng_for("vits-only").integers(0, 1024, 80), device="cuda")
audio = torch.as_tensor(wl.reference.audio_32k.reshape(-1), device="cuda")
ge = torch.randn(1024, device="cuda"); ga = torch.randn(512, device="cuda")
e.set_timing(True)
ms = []
for i in range(n):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    if version == "v2":
        e.vits_decode(txt, sem, ref_audio=audio)
    else:
        e.vits_decode(txt, sem, ge=ge, ge_advanced=ga)
    torch.cuda.synchronize(); ms.append((time.perf_counter() - t0) * 1e3)
print("vits wall ms", [round(x, 3) for x in ms], "device ms", e.timing()[3])
