"""Host-side time per call of the pipelined single-utterance loop (bench.py
step_overlap): where the ~0.4 ms between one decode and the next goes."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from genie_tts_amd import workloads  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
wl = workloads.single()
run = bench.Runner(wl, wl.items, torch.device("cuda", 0), 0)
run.eng.set_vocoder_cus(64)
eng = run.eng
eng.set_timing(len(sys.argv) > 1 and sys.argv[1] == "timing")
utt = (run.d_ref, run.d_txt[0], run.d_ref_bert, run.d_bert[0], run.d_ssl, wl.items[0].force_steps)
T = {k: [] for k in ("prefetch", "generate", "wait", "async", "step")}
pending = None
for i in range(40):
    t0 = time.perf_counter()
    eng.t2s_prefetch(utt, run.sp)
    t1 = time.perf_counter()
    sems = eng.t2s_generate([utt], run.sp)
    t2 = time.perf_counter()
    if pending is not None:
        eng.vits_wait()
    t3 = time.perf_counter()
    pending = eng.vits_decode_async(dict(text_seq=run.d_txt[0], pred_semantic=sems[0], noise_seed=1,
                                         ref_audio=run.d_audio))
    t4 = time.perf_counter()
    if i >= 5:
        for k, v in zip(T, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0)):
            T[k].append(v * 1e3)
        T.setdefault("decode_dev", []).append(eng.timing()[2])
eng.vits_wait()
print({k: round(float(np.median(v)), 4) for k, v in T.items()})
