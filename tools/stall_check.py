"""Vocoder kernels stalled behind the persistent decode, from a rocprofv3 --kernel-trace
database (r05u reading): per MRF-conv shape, the median and max duration and the durations
of the calls that overlap a k_decode_persist* launch.  Usage: python tools/stall_check.py DIR"""
import glob
import sqlite3
import sys

import numpy as np

db = sqlite3.connect(glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0])
rows = list(db.execute("select name, start, end from kernels"))
dec = [(s, e) for n, s, e in rows if "k_decode_persist" in n]
print("## decode launches (ms):", [round((e - s) / 1e6, 2) for s, e in dec])
shapes = sorted({n for n, _, _ in rows if "k_conv_h" in n or "k_mrf_pair" in n})
worst = 0.0
for sh in shapes:
    d = [(s, e) for n, s, e in rows if n == sh]
    dur = np.array([(e - s) / 1e3 for s, e in d])
    med = float(np.median(dur))
    over = [round((e - s) / 1e3, 1) for s, e in d if any(s < de and e > ds for ds, de in dec)]
    worst = max(worst, max(over) / med if over else 0.0)
    print(f"## {sh[sh.find('<'):sh.find('>') + 1] or sh[:60]}: {len(d)} calls, median {med:.1f} us, "
          f"max {dur.max():.1f} us; overlapping a decode launch: {over}")
print(f"## worst overlapping call / its shape's median: {worst:.2f}")
