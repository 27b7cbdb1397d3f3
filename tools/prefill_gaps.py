"""Kernel-level timeline of one utterance's encode + prefill in the sequential mode
(every CU, no vocoder overlap), from a rocprofv3 --kernel-trace CSV: for the last
persistent decode launch, the kernels since the previous decode's last kernel, their
summed busy time and the span (busy + gaps).  Usage:
  rocprofv3 --kernel-trace --output-format csv -d DIR -o t -- python3 bench.py --vocoder-cus 0 ...
  python tools/prefill_gaps.py DIR"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
dec = [i for i, r in enumerate(rows) if "k_decode_persist1" in r[2]]
i1 = dec[-1]
# the encode + prefill kernels: walk back from the decode over the T2S kernels
t2s = ("gemm", "attn_flash", "layernorm", "k_ln_rows", "audio_embed", "text_embed", "k_seq_init", "k_fill_row",
       "k_sumsq", "k_argmin", "k_ssl_im2col", "k_gemv", "k_sample", "k_kv", "k_prompt", "k_bias")
j = i1 - 1
while j >= 0 and not any(k in rows[j][2] for k in t2s):   # copies / slot moves just before the launch
    j -= 1
while j >= 0 and (any(k in rows[j][2] for k in t2s) or "Buffer" in rows[j][2]):
    j -= 1
seg = rows[j + 1:i1]
busy = sum(e - s for s, e, _ in seg)
span = (seg[-1][1] - seg[0][0]) if seg else 0
print(f"kernels {len(seg)}  busy {busy / 1e3:.1f} us  span {span / 1e3:.1f} us  gaps {(span - busy) / 1e3:.1f} us")
by = {}
for s, e, n in seg:
    k = n.split("(")[0][-48:]
    c, t = by.get(k, (0, 0))
    by[k] = (c + 1, t + e - s)
for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1]):
    print(f"{k:50s} {c:4d} {t / 1e3:9.1f} us  avg {t / c / 1e3:6.2f}")
for s_, e_, n_ in rows[max(0, i1 - 12):i1]:
    print("  tail:", n_[:70], (e_ - s_) / 1e3)
print("first/last:", seg[0][2][:60] if seg else None, "|", seg[-1][2][:60] if seg else None)
