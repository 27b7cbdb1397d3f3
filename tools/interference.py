"""Which concurrent work slows the pipelined decode: the stream of bench.py with the
prefetch and/or the vocoder switched off (decode phase = events around the kernel)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from genie_tts_amd import workloads  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
wl = workloads.single()
run = bench.Runner(wl, wl.items, torch.device("cuda", 0), 0)
eng = run.eng
eng.set_vocoder_cus(64)
eng.set_timing(True)
utt = (run.d_ref, run.d_txt[0], run.d_ref_bert, run.d_bert[0], run.d_ssl, wl.items[0].force_steps)
for pf, voc in ((True, True), (False, True), (True, False), (False, False), (True, True)):
    n = 30
    dec = []
    if pf:
        eng.t2s_prefetch(utt, run.sp)
    eng.t2s_generate_start(utt, run.sp)
    pending = None
    for i in range(n):
        if i + 1 < n:
            if pf:
                eng.t2s_prefetch(utt, run.sp)
            eng.t2s_generate_start(utt, run.sp)
        sem = eng.t2s_generate_finish()
        dec.append(eng.timing()[2])
        if pending is not None:
            eng.vits_wait()
            pending = None
        if voc:
            pending = eng.vits_decode_async(dict(text_seq=run.d_txt[0], pred_semantic=sem, noise_seed=1,
                                                 ref_audio=run.d_audio))
    if pending is not None:
        eng.vits_wait()
    print(f"prefetch={pf} vocoder={voc}: decode median {np.median(dec[3:]):.3f} ms", flush=True)
