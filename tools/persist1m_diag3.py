"""persist1m deviation probe 3: input 62 of the pm64 set in several pairings and with a
prefetch delay (option pf_delay) that shifts the kernel's timing."""
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
    inp = lambda i: t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm64_{i}")
    sp = make_sampler(force_steps=4)
    out = {"single": e.t2s_generate([inp(62)], sp)[0].tolist()}
    for name, idx in [("62,62", [62, 62]), ("0,62", [0, 62]), ("62,0", [62, 0]), ("62,63", [62, 63])]:
        res = e.t2s_generate([inp(i) for i in idx], sp)
        out[name] = [res[k].tolist() for k, i in enumerate(idx) if i == 62]
    for d in (4, 32):
        e.set_option("pf_delay", d)
        out[f"62,0 pf_delay {d}"] = e.t2s_generate([inp(62), inp(0)], sp)[0].tolist()
    e.set_option("pf_delay", 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
