"""Debug-build diagnosis (tools/build_dbg.sh, GENIE_ENGINE_LIB=genie_tts_amd/_lib/alt_dbg/...):
q and the head output of every head at step 1, layers 0..7, for input 62 of the pm64 set,
from a single launch (persist1), the multi-sequence kernel ([62, 0]) and the batched kernel
([62, 0]): the first (layer, head) where they differ."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from genie_tts_amd.engine import Engine, make_sampler
    from tests.common import character, t2s_inputs
    w = character("v2")
    e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
    e.set_option("persist", 1)
    e.set_option("ptrace", 1)
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    e.set_option("knob3", mode)
    e.set_option("persistm_min_b", 2)
    inp = lambda i: t2s_inputs(R=10 + 3 * i, S=8 + 2 * i, H=30 + 6 * i, tag=f"pm64_{i}")
    sp = make_sampler(force_steps=4)
    dumps = {}
    for name, idx, pm in (("single", [62], 1), ("p1m", [62, 0], 0), ("pm", [62, 0], 1)):
        e.set_option("persistm", pm)
        toks = e.t2s_generate([inp(i) for i in idx], sp)[0].tolist()
        raw = e.ptrace().reshape(-1).view(np.float32)[:8192]
        tr = raw[:5048].copy() if mode == 12 else raw.reshape(8, 16, 64).copy() if mode == 7 else np.concatenate([raw[:2048].reshape(16, 128), raw[2048:2080].reshape(16, 2)], 1) if mode >= 10 \
            else raw.reshape(16, 512).copy()
        dumps[name] = (toks, tr)
    out = {k: v[0] for k, v in dumps.items()}
    for a_, b_ in (("single", "p1m"), ("single", "pm")):
        A, B = dumps[a_][1], dumps[b_][1]
        diff = []
        if mode == 12:
            d = np.abs(A - B)
            out[f"{a_} vs {b_}"] = {"mfma": float(d[:64].max()), "v": float(d[64:576].max()), "A": float(d[576:1088].max()),
                                    "ffB": float(d[1088:1600].max()), "v_n1w_now": float(d[1600:2112].max()),
                                    "hi": float(d[2112:2624].max()), "un_at_gather": float(d[3000:3512].max()),
                                    "hi_at_gather": float(d[3512:4024].max()), "v_at_gather": float(d[4024:4536].max()),
                                    "n1w_at_gather": float(d[4536:5048].max()),
                                    "examples": [[int(c), float(A[3000 + c]), float(A[3512 + c]), float(B[3512 + c])]
                                                 for c in np.nonzero(d[3512:4024])[0][:4]],
                                    "A_vs_vn1w_now": [float(np.abs(A[576:1088] - A[1600:2112]).max()),
                                                      float(np.abs(B[576:1088] - B[1600:2112]).max())]}
            continue
        if mode != 7:
            d = np.abs(A - B)
            out[f"{a_} vs {b_}"] = {"max": float(d.max()), "rows_differing": [int(x) for x in np.nonzero(d.max(1))[0]],
                                    "cols_differing_row0": int((d[0] > 0).sum())}
            if mode >= 10:   # columns 128, 129: the LN1 mean / rden of each slice's workgroup
                out[f"{a_} vs {b_}"]["stats_differ"] = bool(d[:, 128:].max() > 0)
                out[f"{a_} vs {b_}"]["f_max_diff"] = float(d[:, :128].max())
            continue
        for l in range(8):
            for h in range(16):
                dq = float(np.abs(A[l, h, :32] - B[l, h, :32]).max())
                do = float(np.abs(A[l, h, 32:] - B[l, h, 32:]).max())
                if dq > 0 or do > 0:
                    diff.append((l, h, dq, do))
        out[f"{a_} vs {b_}"] = {"n_diff": len(diff), "first": diff[:6]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
