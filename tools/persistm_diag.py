"""Diagnose a persistm / persist1m token mismatch: the B = 64 case of
tests/test_persistm_gpu.py (tags pm64_i, 22 forced steps): persistm (x3), persist1m,
per-step graphs and single launches for the sequences that differ."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from genie_tts_amd.engine import Engine, make_sampler
    from tests.common import character, t2s_inputs
    w = character("v2")
    e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
    e.set_option("persist", 1)
    e.set_option("persistm_min_b", 2)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm{B}_{i}") for i in range(B)]
    sp = make_sampler(force_steps=22)
    runs = {}
    e.set_option("persistm", 1)
    for k in range(3):
        runs[f"pm{k}"] = [x.tolist() for x in e.t2s_generate(inps, sp)]
    e.set_option("persistm", 0)
    runs["p1m"] = [x.tolist() for x in e.t2s_generate(inps, sp)]
    e.set_option("persist", 0)
    runs["graph"] = [x.tolist() for x in e.t2s_generate(inps, sp)]
    e.set_option("persist", 1)
    e.set_option("persistm", 1)
    bad = sorted({i for i in range(B) for k in runs if runs[k][i] != runs["p1m"][i]})
    out = {"bad": bad}
    for i in bad[:6]:
        single = e.t2s_generate([inps[i]], sp)[0].tolist()
        out[str(i)] = {k: runs[k][i][:6] for k in runs}
        out[str(i)]["single"] = single[:6]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
