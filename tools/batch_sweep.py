"""T2S generate time vs batch size (B = 1 .. 64) on one GPU: V2 synthetic character, the
single workload's utterance repeated B times (R=48, S=45, H=264, 81 forced loop steps),
greedy.  Prints one JSON line: ms per generate and ms per utterance per decode path, so the
engine's path choice and a batching front end's policy can be read off it.
Usage: python tools/batch_sweep.py [--compare]  (--compare: also the per-step graph path
for B > 8, i.e. with option persist1m = 0)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    eng = Engine(synth.synthetic_character("v2"), "v2")
    eng.set_option("persist", 1)
    T = lambda a: torch.as_tensor(a, device="cuda")
    utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
           it.force_steps)
    sp = make_sampler()
    out = {}
    def timed(parts):
        for p in parts:
            eng.t2s_generate([utt] * p, sp)
        torch.cuda.synchronize()
        n = 5
        t0 = time.perf_counter()
        for _ in range(n):
            for p in parts:
                eng.t2s_generate([utt] * p, sp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    compare = "--compare" in sys.argv
    for B in (1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 24, 32, 40, 48, 56, 64):
        ms = timed([B])
        out[B] = {"ms": round(ms, 2), "ms_per_utt": round(ms / B, 3)}
        if compare and B > 8:   # the per-step graph path at the same B
            eng.set_option("persist1m", 0)
            out[B]["graphs_ms"] = round(timed([B]), 2)
            eng.set_option("persist1m", 1)
        print(B, out[B], file=sys.stderr, flush=True)
    print(json.dumps({"t2s_generate_vs_batch": out, "steps": it.force_steps}))
    eng.close()


if __name__ == "__main__":
    main()
