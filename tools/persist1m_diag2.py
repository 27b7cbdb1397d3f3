"""persist1m on [62, 0] of the pm64 set vs a single launch of 62, under layer-group counts
(GENIE_PERSIST_GROUPS is read per launch) and step counts: where does it deviate?"""
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
    out = {}
    for steps in (4,):
        sp = make_sampler(force_steps=steps)
        single = e.t2s_generate([inps[62]], sp)[0].tolist()
        row = {"single": single}
        row["p1m"] = e.t2s_generate([inps[62], inps[0]], sp)[0].tolist()
        e.set_option("knob0", 1)   # greedy through the sampler workgroups instead of the fused step end
        row["p1m_knob0"] = e.t2s_generate([inps[62], inps[0]], sp)[0].tolist()
        row["single_knob0"] = e.t2s_generate([inps[62]], sp)[0].tolist()
        e.set_option("knob0", 0)
        e.set_option("persist", 0)
        row["graph"] = e.t2s_generate([inps[62], inps[0]], sp)[0].tolist()
        e.set_option("persist", 1)
        e.set_option("persistm", 1)
        e.set_option("persistm_min_b", 2)
        row["persistm"] = e.t2s_generate([inps[62], inps[0]], sp)[0].tolist()
        e.set_option("persistm", 0)
        out[f"steps{steps}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
