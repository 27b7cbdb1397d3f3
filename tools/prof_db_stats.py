"""Per-kernel stats (calls, total/avg us, grid) from a rocprofv3 rocpd .db file.
Usage: python tools/prof_db_stats.py <results.db> [top]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
agg = collections.defaultdict(lambda: [0, 0.0, set()])
tot = 0.0
for kid, s, e, gx, wx in c.execute("select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch"):
    a = agg[names.get(kid, str(kid)).split("(")[0]]
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2].add(gx // max(wx, 1))
    tot += (e - s) / 1e3
print(f"{'kernel':48s} {'calls':>7s} {'total_ms':>9s} {'avg_us':>8s} {'pct':>6s}  blocks")
for k, (n, us, g) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{k[:48]:48s} {n:7d} {us/1e3:9.2f} {us/n:8.2f} {100*us/tot:6.2f}  {sorted(g)[:4]}")
print(f"total kernel time {tot/1e3:.2f} ms")
