"""Per-phase kernel time vs wall span of the LAST utterance in a rocprofv3 db
(bench.py configs[1]): prefill = kernels before the persistent decode launch,
VITS = kernels after it.  Usage: python tools/utt_timeline.py DB [top]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = db.execute("select name, start, end, duration, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
dec = [i for i, r in enumerate(rows) if "k_decode_persist" in r[0]]
last, prev = dec[-1], dec[-2]
# the utterance: after the previous utterance's VITS (first kernel after prev decode that is an encoder kernel)
# -> take the kernels between prev decode's following VITS end and this decode: find the largest gap
seg = rows[prev + 1:last]
gaps = [(seg[i + 1][1] - seg[i][2], i) for i in range(len(seg) - 1)]
cut = max(gaps)[1] + 1
pre = seg[cut:]
vits = rows[last + 1:]


def report(name, ks):
    span = (ks[-1][2] - ks[0][1]) / 1000
    busy = sum(k[3] for k in ks) / 1000
    print(f"== {name}: {len(ks)} kernels, wall span {span:.1f} us, kernel time {busy:.1f} us, gaps {span - busy:.1f} us")
    agg = collections.OrderedDict()
    for k in ks:
        key = (k[0].replace("void ", "").replace("gsv::", "").replace("(anonymous namespace)::", "").split("(")[0],
               k[4] // max(1, k[7]), k[5], k[6])
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += k[3] / 1000
    for kk, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {kk[0][:40]:40s} grid=({kk[1]},{kk[2]},{kk[3]}) n={v[0]:3d} total={v[1]:8.1f}us avg={v[1] / v[0]:7.1f}")


report("encode+prefill", pre)
print(f"== decode: {rows[last][3] / 1000:.1f} us")
report("vits", vits)
