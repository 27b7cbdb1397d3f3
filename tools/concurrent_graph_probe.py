"""Probe: is a batch-64 decode faster as N concurrent per-step-graph decodes of 64 / N
sequences (one engine per sub-batch, each on its own stream, driven from its own host
thread) than as one persistent multi-sequence launch?  V2 synthetic character, the single
workload's utterance, 81 forced steps, greedy.  Prints one JSON line of ms per 64 utterances.
Usage: python tools/concurrent_graph_probe.py [total_B]"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    wl = workloads.single()
    ref, it = wl.reference, wl.items[0]
    ch = synth.synthetic_character("v2")
    engines = [Engine(ch, "v2") for _ in range(4)]
    for e in engines:
        e.set_option("persist", 1)
    T = lambda a: torch.as_tensor(a, device="cuda")
    utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
           it.force_steps)
    sp = make_sampler()
    streams = [torch.cuda.Stream() for _ in range(4)]
    reps = 3
    out = {"B": total, "steps": it.force_steps}
    toks = {}

    def run(n, persist):
        b = total // n
        for e in engines[:n]:
            e.set_option("persist1m", 1 if persist else 0)
        res = [None] * n
        def work(i):   # each thread on its own torch stream: the engines' stream scopes stay unordered
            with torch.cuda.stream(streams[i]):
                res[i] = engines[i].t2s_generate([utt] * b, sp)
        def once():
            th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        once()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            once()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3, res

    # (4 engines x 16 on threads is tools/concurrency_probe.py's case -- r04 failed it with
    # capture errors, fixed in r05 (profiles/r05_concurrency.txt); two persistent launches
    # cannot be co-resident, so this probe only asks whether per-step-graph streams overlap)
    for n, persist in ((1, True), (1, False), (2, False)):
        key = f"{n}x{total // n}_{'persist' if persist else 'graph'}"
        ms, res = run(n, persist)
        out[key] = round(ms, 2)
        toks[key] = res
        print(key, out[key], file=sys.stderr, flush=True)
    # every configuration must produce the same tokens for the same utterance
    first = next(iter(toks.values()))[0][0]
    out["tokens_identical"] = all(np.array_equal(t, first) for res in toks.values() for r in res for t in r)
    print(json.dumps(out))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
