"""Per-shape breakdown of the last utterance's VITS kernels from a rocprofv3 db."""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = db.execute("select name,grid_x,grid_y,grid_z,workgroup_x,duration,start from kernels order by start").fetchall()
last = [i for i, r in enumerate(rows) if "k_sample" in r[0]][-1]
agg = collections.OrderedDict()
tot = 0.0
for r in rows[last + 1:]:
    key = (r[0].split("(")[0].replace("void ", "").replace("gsv::", ""), r[1] // max(1, r[4]), r[2], r[3])
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += r[5] / 1000
    tot += r[5] / 1000
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{k[0]:28s} grid=({k[1]},{k[2]},{k[3]}) n={v[0]:3d} total={v[1]:8.1f}us avg={v[1] / v[0]:7.1f}")
print(f"total {tot:.1f} us over {len(rows) - last - 1} kernels")
