"""Probe: several engines of one process, one host thread each, decoding
B sequences on the per-step graphs at once -- the configuration of gpurun_out/r04o_probe.err
("decode graph capture failed", "encode launch").  Each round uses a sampler no graph was
captured for, so every engine captures while the others launch / capture / synchronise.
Prints per round the errors raised by the threads, whether all tokens agree, and the
engines' graph_fallbacks counters.  GENIE_ENGINE_LIB selects another build (A/B).
Usage: python tools/concurrency_probe.py [engines] [B] [steps] [rounds]"""
import json
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 81
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    ch = synth.synthetic_character("v2")
    engines = [Engine({k: ch[k] for k in ("t2s_encoder", "t2s")}, "v2") for _ in range(n)]
    for e in engines:
        e.set_option("persist1m", 0)
    T = lambda a: torch.as_tensor(a, device="cuda")
    utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)), steps)
    streams = [torch.cuda.Stream() for _ in range(n)]
    want = engines[0].t2s_generate([utt] * B, make_sampler(max_steps=499))
    out = {"engines": n, "B": B, "steps": steps, "lib": os.environ.get("GENIE_ENGINE_LIB", "in-tree"), "rounds": []}
    for r in range(rounds):
        sp = make_sampler(max_steps=450 + r)
        res, errs = [None] * n, []

        def work(i):
            try:
                with torch.cuda.stream(streams[i]):
                    res[i] = engines[i].t2s_generate([utt] * B, sp)
            except Exception as ex:
                errs.append(f"engine {i}: {ex}")

        th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        same = all(x is not None and all(np.array_equal(a, b) for a, b in zip(x, want)) for x in res)
        try:
            fb = [e.counter("graph_fallbacks") for e in engines]
        except Exception:
            fb = None
        out["rounds"].append({"errors": errs, "tokens_identical": same if not errs else None, "graph_fallbacks": fb})
        print(json.dumps(out["rounds"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
