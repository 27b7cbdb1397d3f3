"""Per-launch durations of the last SV call in a rocprofv3 --kernel-trace CSV (order = launch order in sv.hip)."""
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
# last SV call: from the last k_sv_fbank to the last k_sv_pool
i0 = max(i for i, r in enumerate(rows) if "k_sv_fbank" in r[2])
i1 = max(i for i, r in enumerate(rows) if "k_sv_pool" in r[2])
for j, (s, e, n) in enumerate(rows[i0:i1 + 1]):
    print(j, n.split("(")[0][-30:], round((e - s) / 1e3, 1))
