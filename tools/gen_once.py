"""One T2S generate of B copies of the single workload's utterance (81 forced steps),
repeated N times, for a kernel trace of one decode path.
Usage: python tools/gen_once.py B N [persist1m=0|1]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    B, N = int(sys.argv[1]), int(sys.argv[2])
    p1m = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    eng = Engine(synth.synthetic_character("v2"), "v2")
    eng.set_option("persist", 1)
    eng.set_option("persist1m", p1m)
    T = lambda a: torch.as_tensor(a, device="cuda")
    utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
           it.force_steps)
    sp = make_sampler()
    eng.t2s_generate([utt] * B, sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        eng.t2s_generate([utt] * B, sp)
    torch.cuda.synchronize()
    print(f"B={B} persist1m={p1m}: {(time.perf_counter() - t0) / N * 1e3:.2f} ms per generate", flush=True)


if __name__ == "__main__":
    main()
