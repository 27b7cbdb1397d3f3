"""Summarise a rocprofv3 kernel-trace database (per-kernel count / total / avg / min / max in us)."""
import glob
import sqlite3
import sys


def summary(db, top=40, name_filter=None):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rows = c.execute("select * from kernels").fetchall()
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    si, ei = cols.index("start"), cols.index("end")
    agg = {}
    for r in rows:
        n = r[ni]
        if name_filter and name_filter not in n:
            continue
        d = (r[ei] - r[si]) / 1000.0
        a = agg.setdefault(n, [0, 0.0, 1e30, 0.0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(v[1] for v in agg.values())
    out = []
    out.append(f"{'kernel':70s} {'calls':>7s} {'total_us':>11s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'%':>6s}")
    for n, (k, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"{n[:70]:70s} {k:7d} {t:11.1f} {t / k:9.2f} {mn:8.2f} {mx:8.2f} {100 * t / tot:6.2f}")
    out.append(f"TOTAL kernel time {tot:.1f} us over {sum(v[0] for v in agg.values())} dispatches")
    return "\n".join(out)


if __name__ == "__main__":
    path = sys.argv[1]
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    print(summary(dbs[0], name_filter=sys.argv[2] if len(sys.argv) > 2 else None))
