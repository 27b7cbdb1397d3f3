"""Batched decode: the per-step graph path vs the multi-sequence persistent kernel at one
batch size (V2 synthetic character, the single workload's utterance repeated B times, 81
forced steps, greedy).  Prints ms per generate of each path and the prefill alone (a
1-step generate), so the decode time per step can be read off.
Usage: python tools/decode_graph_prof.py B [graph|persist|both] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    which = sys.argv[2] if len(sys.argv) > 2 else "both"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    eng = Engine(synth.synthetic_character("v2"), "v2")
    eng.set_option("persist", 1)
    T = lambda a: torch.as_tensor(a, device="cuda")
    def utt(steps):
        return (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
                steps)
    sp = make_sampler()
    def timed(steps):
        eng.t2s_generate([utt(steps)] * B, sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.t2s_generate([utt(steps)] * B, sp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3
    out = {"B": B, "steps": it.force_steps}
    out["prefill_1step_ms"] = round(timed(1), 2)
    paths = ("graph", "persist") if which == "both" else (which,)
    for p in paths:
        eng.set_option("persist1m", 1 if p == "persist" else 0)
        ms = timed(it.force_steps)
        out[p] = {"ms": round(ms, 2),
                  "decode_ms_per_step": round((ms - out["prefill_1step_ms"]) / (it.force_steps - 1), 4)}
        print(p, out[p], file=sys.stderr, flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
