"""Debug: the test_vits_batch_lanes_match_single items, single calls twice (determinism)
and the batch on lanes (seg_vocoder 0) vs single; prints mismatch counts and where."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from genie_tts_amd import synth
from genie_tts_amd.engine import Engine
from tests.common import character

w = character("v2")
e = Engine({k: w[k] for k in ("t2s_encoder", "t2s", "vits") if k in w}, "v2")
kw = dict(ref_audio=synth.synth_ref_audio(32000 * 2 + 1234))
items = []
for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9), (47, 31), (26, 18), (40, 40)]):
    txt = synth.synth_phones(S, f"vb{i}")
    sem = ((np.arange(G, dtype=np.int64) * (7 + i) + 3 * i) % 1024).reshape(1, 1, G)
    it = dict(text_seq=txt, pred_semantic=sem, **kw)
    if i % 3 == 1:
        it["noise_seed"] = 1000 + i
    elif i % 3 == 2:
        it["eps"] = synth.rng_for(f"vbe{i}").standard_normal((1, 192, 2 * G)).astype(np.float32)
    items.append(it)
# stale data in every workspace first: longer utterances through single calls and the lanes
big = [dict(text_seq=synth.synth_phones(30, f"bg{i}"),
            pred_semantic=((np.arange(90, dtype=np.int64) * (3 + i)) % 1024).reshape(1, 1, 90),
            eps=(synth.rng_for(f"bge{i}").standard_normal((1, 192, 180)) * (1e6 if i == 1 else 1.0)).astype(np.float32),
            **kw) for i in range(6)]
e.set_option("seg_vocoder", 0)
e.vits_decode_batch(big)
for it in big[:2]:
    e.vits_decode(it["text_seq"], it["pred_semantic"], eps=it["eps"], **kw)
e.set_option("seg_vocoder", 1)
one = lambda it: e.vits_decode(it["text_seq"], it["pred_semantic"], eps=it.get("eps"), noise_seed=it.get("noise_seed"),
                               **kw).cpu().numpy()
s1 = [one(it) for it in items]
s2 = [one(it) for it in items]
print("reruns", e.counter("vits_f32_reruns"))
for i in range(len(items)):
    d = np.nonzero(s1[i] != s2[i])[0]
    print(f"single x2 item {i}: {d.size} differ", d[:5], d[-5:] if d.size else "")
e.set_option("seg_vocoder", 0)
outs = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
print("reruns", e.counter("vits_f32_reruns"))
for i in range(len(items)):
    d = np.nonzero(outs[i] != s1[i])[0]
    print(f"lanes vs single item {i}: {d.size} differ of {s1[i].size}", d[:8], d[-8:] if d.size else "",
          float(np.abs(outs[i] - s1[i]).max()))
    if d.size:   # which output phase / region: samples per frame 640 (10 x 8 x 2 x 2 x 2)
        print("   frames", np.unique(d // 640)[:20], "sample%10", np.unique(d % 10), "n_frames", s1[i].size // 640)

# repeat: the same lanes batch again (stale-state vs deterministic), then one lane (no concurrency)
def cmp(tag, outs):
    for i in range(len(items)):
        d = np.nonzero(outs[i] != s1[i])[0]
        print(f"{tag} item {i}: {d.size} differ", float(np.abs(outs[i] - s1[i]).max()) if d.size else 0.0)
cmp("lanes again", [o.cpu().numpy() for o in e.vits_decode_batch(items)])
e.set_option("vits_lanes", 1)
cmp("one lane", [o.cpu().numpy() for o in e.vits_decode_batch(items)])
e.set_option("vits_lanes", 4)
cmp("lanes after one-lane", [o.cpu().numpy() for o in e.vits_decode_batch(items)])

# host threading vs GPU concurrency: lanes issued by ONE host thread (vits_threads 0), 4 streams
e.set_option("vits_threads", 0)
for r in range(3):
    cmp(f"4 lanes, one issuing thread, rep {r}", [o.cpu().numpy() for o in e.vits_decode_batch(items)])
e.set_option("vits_threads", 1)
for r in range(2):
    cmp(f"4 lanes, thread per lane, rep {r}", [o.cpu().numpy() for o in e.vits_decode_batch(items)])
