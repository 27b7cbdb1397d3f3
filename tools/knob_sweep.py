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
    # step end (8 layer groups): layer 23 FFN (group 7, blocks 240..255) publish at s4, logits
    # workgroups (group 1 FFN, blocks 48..63): s0 start, s1 x_24 formed, s2 logits published;
    # sampler (block 64): s0 woken, s1 logits read, s2 token published; layer 0 of step 9
    # (group 0 attention, blocks 0..15): s0 token known, s1 q/k/v operand ready, s5 published
    def med(b0, b1, i):
        v = (tr[b0:b1, i] - t0) * 10 / 1000.0
        return float(np.median(v))
    print("step end: L23 ffn publish %.2f | logits start %.2f x24 %.2f published %.2f | sampler woke %.2f "
          "logits read %.2f token %.2f | L0(s9) start %.2f operand %.2f attn published %.2f | L1(s9)?" % (
              med(240, 256, 4), med(48, 64, 0), med(48, 64, 1), med(48, 64, 2), med(64, 65, 0), med(64, 65, 1),
              med(64, 65, 2), med(0, 16, 0), med(0, 16, 1), med(0, 16, 5)), flush=True)
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
