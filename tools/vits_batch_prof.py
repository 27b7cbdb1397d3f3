"""batch64's vocoder alone: the 64 sentences' vits_decode_batch (synthetic V2 character,
random semantic tokens of the workload's lengths, Philox noise), timed per call; with
--trace DB (a rocprofv3 kernel-trace database of this run) it splits the last call's wall
time into the per-utterance front part (lanes) and the segmented generator (from the
first conv_pre launch, k_conv1d<7>, to the end).
Usage: python tools/vits_batch_prof.py [N] [--seg 0|1] [--front 0|1] [--opt name=value] [--n sentences]
     | python tools/vits_batch_prof.py --trace DIR
     | python tools/vits_batch_prof.py --convs DIR   (the last call's generator convs in launch order:
       stage, kernel, grid, microseconds -- the MRF convs of a stage are 3 resblocks x 3 dilations x 2)"""
import glob
import os
import sqlite3
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def trace(path):
    db = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    si, ei = cols.index("start"), cols.index("end")
    rows = sorted((r[si], r[ei], r[ni]) for r in c.execute("select * from kernels"))
    # calls are separated by host gaps > 2 ms; take the last call
    calls, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur[-50:]) > 2e6:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    for k, call in enumerate(calls[-3:]):
        t0, t1 = call[0][0], max(r[1] for r in call)
        g0 = next((r[0] for r in call if "k_conv1d<7" in r[2]), t1)
        print(f"call {k}: {len(call)} kernels, wall {(t1 - t0) / 1e6:.2f} ms: front {(g0 - t0) / 1e6:.2f} ms, "
              f"generator {(t1 - g0) / 1e6:.2f} ms")


def convs(path):
    db = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    si, ei = cols.index("start"), cols.index("end")
    gi = [cols.index(k) for k in ("grid_x", "grid_y", "grid_z") if k in cols]
    rows = sorted(c.execute("select * from kernels"), key=lambda r: r[si])
    calls, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[si] - max(x[ei] for x in cur[-50:]) > 2e6:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    call = calls[-1]
    g0 = next(i for i, r in enumerate(call) if "k_conv1d<7" in r[ni])
    stage, tot = -1, {}
    for r in call[g0:]:
        n = r[ni]
        short = n.replace("void ", "").replace("gsv::(anonymous namespace)::", "").replace("gsv::", "").split("(")[0]
        us = (r[ei] - r[si]) / 1e3
        grid = tuple(r[i] for i in gi)
        if "k_conv_h" in short and grid and len(grid) == 3 and grid[2] > 1:
            stage += 1   # the polyphase ConvTranspose (z = phases) opens a stage
        print(f"stage {stage} {short:45s} grid {grid} {us:9.1f} us")
        tot.setdefault((stage, short), []).append(us)
    for (st, k), v in sorted(tot.items()):
        print(f"total stage {st} {k:45s} {len(v):3d} x {sum(v) / len(v):8.1f} us = {sum(v) / 1e3:7.2f} ms")


def allk(path):
    """Every kernel of the last call in launch order: duration, the gap since the previous end."""
    db = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    si, ei = cols.index("start"), cols.index("end")
    rows = sorted(c.execute("select * from kernels"), key=lambda r: r[si])
    calls, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[si] - max(x[ei] for x in cur[-50:]) > 2e6:
            calls.append(cur)
            cur = []
        cur.append(r)
    calls.append(cur)
    call = calls[-1]
    busy, gaps, prev, agg = 0.0, 0.0, None, {}
    for r in call:
        short = r[ni].replace("void ", "").replace("gsv::(anonymous namespace)::", "").replace("gsv::", "").split("(")[0]
        us = (r[ei] - r[si]) / 1e3
        gap = (r[si] - prev) / 1e3 if prev is not None else 0.0
        print(f"{short:45s} {us:9.1f} us  gap {gap:7.1f}")
        busy += us
        gaps += max(gap, 0.0)
        prev = max(prev or 0, r[ei])
        a = agg.setdefault(short, [0, 0.0])
        a[0] += 1
        a[1] += us
    print(f"# {len(call)} kernels, wall {(max(r[ei] for r in call) - call[0][si]) / 1e3:.1f} us, "
          f"bodies {busy:.1f} us, gaps {gaps:.1f} us")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"total {k:45s} {n:4d} x {us / n:8.1f} us = {us:8.1f} us")


def main():
    if "--all" in sys.argv:
        return allk(sys.argv[sys.argv.index("--all") + 1])
    if "--convs" in sys.argv:
        return convs(sys.argv[sys.argv.index("--convs") + 1])
    if "--trace" in sys.argv:
        return trace(sys.argv[sys.argv.index("--trace") + 1])
    import numpy as np
    import torch
    from genie_tts_amd import synth, workloads
    from genie_tts_amd.engine import Engine
    n_calls = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
    wl = workloads.batch64()
    eng = Engine(synth.synthetic_character("v2"), "v2")
    if "--seg" in sys.argv:
        eng.set_option("seg_vocoder", int(sys.argv[sys.argv.index("--seg") + 1]))
    if "--front" in sys.argv:
        eng.set_option("seg_front", int(sys.argv[sys.argv.index("--front") + 1]))
    for i, a in enumerate(sys.argv):   # --opt name=value: any engine option (A/B of a vocoder path)
        if a == "--opt":
            k, v = sys.argv[i + 1].split("=")
            eng.set_option(k, int(v))
    if "--n" in sys.argv:   # the first n sentences only (n = 1: one utterance, the single-call path)
        wl.items = wl.items[:int(sys.argv[sys.argv.index("--n") + 1])]
    ref = wl.reference
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device="cuda")
    ge = eng.ref_encode(T(ref.audio_32k.reshape(-1)))
    r = np.random.default_rng(5)
    items = [dict(text_seq=T(it.text_seq.reshape(-1)), pred_semantic=T(r.integers(0, 1024, it.tokens)),
                  noise_seed=0x5EED + i, ge=ge) for i, it in enumerate(wl.items)]
    for k in range(n_calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.vits_decode_batch(items)
        torch.cuda.synchronize()
        print(f"call {k}: {(time.perf_counter() - t0) * 1e3:.2f} ms for {len(items)} utterances", flush=True)
        time.sleep(0.01)   # a host gap between calls (the trace splitter keys on it)


if __name__ == "__main__":
    main()
