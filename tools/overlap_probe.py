"""Phase times of one utterance with the vocoder_cus stream split set but no
overlap: T2S alone (encode, prefill, decode) and the vocoder alone on its CUs."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from genie_tts_amd import synth, workloads  # noqa: E402
from genie_tts_amd.engine import Engine, make_sampler  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
wl = workloads.single()
it, ref = wl.items[0], wl.reference
eng = Engine(synth.synthetic_character("v2"), "v2")
eng.set_option("persist", 1)
d = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
rs, ssl, au, txt = d(ref.ref_seq.reshape(-1)), d(ref.ssl.reshape(768, -1)), d(ref.audio_32k.reshape(-1)), d(it.text_seq.reshape(-1))
sp = make_sampler(top_k=wl.top_k, greedy=wl.greedy)
eng.set_timing(True)
if K:
    eng.set_vocoder_cus(K)
res = {"K": K}
for mode in ("t2s", "vits"):
    ts = []
    for i in range(8):
        sems = eng.t2s_generate([(rs, txt, None, None, ssl, it.force_steps)], sp)
        tm = eng.timing()
        if mode == "t2s":
            ts.append(tm[:3])
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if K:
            eng.vits_decode_async(dict(text_seq=txt, pred_semantic=sems[0], noise_seed=1, ref_audio=au))
            eng.vits_wait()
        else:
            eng.vits_decode(txt, sems[0], ref_audio=au, noise_seed=1)
        torch.cuda.synchronize()
        ts.append([eng.timing()[3], (time.perf_counter() - t0) * 1e3])
    res[mode] = np.mean(np.asarray(ts[2:]), axis=0).round(3).tolist()
print(json.dumps(res), flush=True)
