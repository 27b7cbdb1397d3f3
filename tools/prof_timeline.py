"""Print the kernel timeline (start offset, duration, gap) of a window of dispatches."""
import glob
import sqlite3
import sys

path = sys.argv[1]
start_name = sys.argv[2] if len(sys.argv) > 2 else "k_decode_embed"
count = int(sys.argv[3]) if len(sys.argv) > 3 else 80
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 40
db = glob.glob(path + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
si, ei = cols.index("start"), cols.index("end")
rows = sorted(c.execute("select * from kernels").fetchall(), key=lambda r: r[si])
idx = [i for i, r in enumerate(rows) if start_name in r[ni]]
i0 = idx[min(skip, len(idx) - 1)]
t0 = rows[i0][si]
prev_end = t0
tot_gap = tot_k = 0.0
for r in rows[i0:i0 + count]:
    d = (r[ei] - r[si]) / 1000
    g = (r[si] - prev_end) / 1000
    tot_gap += max(g, 0)
    tot_k += d
    print(f"{(r[si]-t0)/1000:9.2f} {d:8.2f} gap {g:6.2f}  {r[ni][:80]}")
    prev_end = r[ei]
print(f"kernels {tot_k:.1f} us, gaps {tot_gap:.1f} us")
