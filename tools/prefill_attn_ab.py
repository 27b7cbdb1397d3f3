"""Packed prefill of batch64's 64 sentences alone (one forced loop step), to A/B the
packed-prefill attention kernels in isolation: GENIE_PACKED_ROWLANE=1 (k_attn_rowlane) or
0 (k_attn_flash over 16-row tiles), GENIE_ATTN_MFMA=1 (k_attn_mfma).  Prints ms per
generate and the tokens' hash (equal across the f32 kernels).
Usage: GENIE_PACKED_ROWLANE=0 python tools/prefill_attn_ab.py"""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    wl = workloads.batch64()
    ref = wl.reference
    e = Engine(synth.synthetic_character("v2"), "v2")
    T = lambda a: torch.as_tensor(a, device="cuda")
    utts = [(T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)), 1)
            for it in wl.items]
    sp = make_sampler()
    out = e.t2s_generate(utts, sp)
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        out = e.t2s_generate(utts, sp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    h = hashlib.sha1(b"".join(o.tobytes() for o in out)).hexdigest()[:16]
    print(json.dumps({"rowlane": os.environ.get("GENIE_PACKED_ROWLANE", "1"),
                      "mfma": os.environ.get("GENIE_ATTN_MFMA", "0"), "ms_per_generate": round(ms, 2),
                      "tokens_sha": h}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
