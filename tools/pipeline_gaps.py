"""Pipelined bench (vocoder overlap + T2S prefetch) from a rocprofv3 kernel-trace
database: the idle time of the decode CUs between one persistent decode launch
and the next, what ran on the engine stream in that gap, and how long the
vocoder + prefetch work beside each decode took.  Usage: python tools/pipeline_gaps.py DB"""
import collections
import sqlite3
import sys

import numpy as np

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
rows = db.execute("select * from kernels order by start").fetchall()
ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
si, ei = cols.index("start"), cols.index("end")
qcol = next((c for c in ("stream_id", "queue_id") if c in cols), None)
dec = [i for i, r in enumerate(rows) if "k_decode_persist" in r[ni]]
gaps, between, beside = [], collections.Counter(), []
for a, b in zip(dec[:-1], dec[1:]):
    d0, d1 = rows[a], rows[b]
    gaps.append((d1[si] - d0[ei]) / 1000)
    for r in rows[a + 1:b]:
        if r[si] >= d0[ei]:
            between[r[ni].split("(")[0][-48:]] += 1
    side = [r for r in rows[a + 1:b] if r[si] < d0[ei]]
    if side:
        beside.append(((max(r[ei] for r in side) - min(r[si] for r in side)) / 1000, len(side),
                       (d0[ei] - d0[si]) / 1000))
g = np.asarray(gaps[2:]) if len(gaps) > 4 else np.asarray(gaps)
print(f"decode launches {len(dec)}; gap decode end -> next decode start (us): "
      f"median {np.median(g):.1f} mean {g.mean():.1f} min {g.min():.1f} max {g.max():.1f}")
print("kernels started in the gaps (all gaps):")
for n, c in between.most_common(12):
    print(f"  {c:5d}  {n}")
if beside:
    bs = np.asarray([x[0] for x in beside[2:] or beside])
    print(f"work beside a decode (vocoder + prefetch span, us): median {np.median(bs):.1f}; "
          f"kernels per decode {int(np.median([x[1] for x in beside]))}; decode {np.median([x[2] for x in beside]):.1f} us")
print("stream/queue column:", qcol)
