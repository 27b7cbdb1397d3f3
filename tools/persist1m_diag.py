"""persist1m vs single launches on subsets of the B = 64 set of tests/test_persistm_gpu.py
(tags pm64_i) that hold sequence 62, and the same with GENIE_PERSIST_GROUPS variations."""
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
    e.set_option("persistm", 0)
    inps = [t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm64_{i}") for i in range(64)]
    sp = make_sampler(force_steps=22)
    single = {i: e.t2s_generate([inps[i]], sp)[0].tolist() for i in range(48, 64)}
    out = {}
    for name, idx in [("64", list(range(64))), ("48-63", list(range(48, 64))), ("60-63", list(range(60, 64))),
                      ("62-63", [62, 63]), ("62,0", [62, 0]), ("56-63", list(range(56, 64)))]:
        res = []
        for rep in range(2):
            got = [x.tolist() for x in e.t2s_generate([inps[i] for i in idx], sp)]
            res.append([i for k, i in enumerate(idx) if i in single and got[k] != single[i]])
        out[name] = res
        print(name, res, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
