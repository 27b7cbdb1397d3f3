"""Decode time of the single-sequence persistent kernel under tuning variants
(engine options knob0..knob3, pf=pf_delay), plus the two-layer phase trace and the shader
clock of the default path.  Usage: python tools/knob_sweep.py "k1=1,k0=1" "k1=1,k0=4" ...
(each argument one variant; the default path is always measured first and last)."""
import sys
sys.path.insert(0, ".")
import numpy as np
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine, make_sampler

w = synth.synthetic_character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s")}, "v2")
ref = synth.synth_phones(48, "r"); txt = synth.synth_phones(45, "t"); ssl = synth.synth_ssl(264)
e.set_timing(True)
base = None


def run(knobs, reps=4):
    for i in range(4):
        e.set_option(f"knob{i}", knobs.get(i, 0))
    e.set_option("pf_delay", knobs.get("pf", 0))
    ts, toks = [], None
    for _ in range(reps):
        out = e.t2s_generate([(ref, txt, None, None, ssl)], make_sampler(force_steps=81))
        ts.append(e.timing()[2])
        toks = out[0]
    return min(ts), float(np.median(ts)), toks


def phase_trace():
    e.set_option("ptrace", 1)
    run({}, reps=2)
    tr = e.ptrace().astype(np.int64)
    e.set_option("ptrace", 0)
    t0 = tr[128:144, 0].min()
    for nm, b in (("attn12", 128), ("ffn12", 144), ("attn13", 160), ("ffn13", 176)):
        t = (tr[b:b + 16, :8] - t0) * 10 / 1000.0
        print(f"{nm:6s} " + "  ".join(f"s{i} {t[:, i].min():6.2f}/{np.median(t[:, i]):6.2f}/{t[:, i].max():6.2f}"
                                    for i in range(8) if -1e5 < t[:, i].max() < 1e5), flush=True)
    # shader clock: memtime ticks / realtime ticks (100 MHz) between the first and last stamp of a block
    for b in (128, 144):
        rt, st = tr[b, :8], tr[b, 8:16]
        m = (rt > 0) & (st > 0)
        idx = np.where(m)[0]
        if len(idx) >= 2:
            i0, i1 = idx.min(), idx.max()
            print(f"clock block {b}: {(st[i1] - st[i0]) / max(1, rt[i1] - rt[i0]) * 100:.0f} MHz", flush=True)


base = run({})
print(f"default: min {base[0]:.3f} ms median {base[1]:.3f}", flush=True)
phase_trace()
for arg in sys.argv[1:]:
    kn = {}
    for kv in arg.split(","):
        k, v = kv.split("=")
        kn["pf" if k == "pf" else int(k[1:])] = int(v)
    r = run(kn)
    same = bool(np.array_equal(r[2], base[2]))
    print(f"{arg:20s}: min {r[0]:.3f} ms median {r[1]:.3f}  tokens {'same' if same else 'DIFFER'}", flush=True)
r = run({})
print(f"default again: min {r[0]:.3f} ms median {r[1]:.3f}", flush=True)
