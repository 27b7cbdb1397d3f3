"""Batched persistent decode (k_decode_persistm, t2s_persistm.hip) against the
multi-sequence kernel (k_decode_persist1m): tokens of both at several B (greedy and
top-k sampled), then ms per generate of the bench utterance x B for both paths.
Usage: python tools/persistm_probe.py [check|time|both]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine, make_sampler
    from tests.common import character, t2s_inputs
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    out = {}
    if mode in ("check", "both"):
        w = character("v2")
        e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
        e.set_option("persistm_min_b", 2)
        res = []
        for B, sp in [(2, make_sampler(force_steps=22)), (5, make_sampler(force_steps=22)),
                      (16, make_sampler(force_steps=22)), (40, make_sampler(force_steps=22)),
                      (64, make_sampler(force_steps=22)),
                      (6, make_sampler(top_k=15, greedy=False, seed=99, force_steps=20))]:
            inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"m{B}_{i}") for i in range(B)]
            n0 = e.counter("persist_launches")
            e.set_option("persistm", 1)
            a = [x.tolist() for x in e.t2s_generate(inps, sp)]
            e.set_option("persistm", 0)
            b = [x.tolist() for x in e.t2s_generate(inps, sp)]
            e.set_option("persistm", 1)
            bad = [i for i in range(B) if a[i] != b[i]]
            res.append({"B": B, "greedy": sp.greedy, "mismatch": bad[:8], "n_bad": len(bad),
                        "launches": e.counter("persist_launches") - n0, "timeouts": e.counter("persist_timeouts"),
                        "f16_reruns": e.counter("persist1_f16_reruns")})
            print(json.dumps(res[-1]), file=sys.stderr, flush=True)
        out["check"] = res
        e.close()
    if mode in ("time", "both"):
        wl = workloads.single()
        ref, it = wl.reference, wl.items[0]
        e = Engine(synth.synthetic_character("v2"), "v2")
        e.set_option("persistm_min_b", 2)
        T = lambda a: torch.as_tensor(a, device="cuda")
        utt = (T(ref.ref_seq.reshape(-1)), T(it.text_seq.reshape(-1)), None, None, T(ref.ssl.reshape(768, -1)),
               it.force_steps)
        sp = make_sampler()
        rows = []
        knobs = [int(x) for x in os.environ.get("PM_KNOB2", "0").split(",")]
        for B in [int(x) for x in os.environ.get("PM_BS", "8,16,32,48,64").split(",")]:
            row = {"B": B}
            for pm in [(1, k) for k in knobs] + [(0, 0)]:
                pm, k2 = pm
                e.set_option("knob2", k2)
                e.set_option("persistm", pm)
                e.t2s_generate([utt] * B, sp)
                torch.cuda.synchronize()
                n = 4
                t0 = time.perf_counter()
                for _ in range(n):
                    e.t2s_generate([utt] * B, sp)
                torch.cuda.synchronize()
                row[(f"persistm_split{k2}" if len(knobs) > 1 else "persistm") if pm else "persist1m"] = \
                    round((time.perf_counter() - t0) / n * 1e3, 2)
            e.set_option("knob2", 0)
            rows.append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
        out["time_ms_per_generate"] = rows
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
