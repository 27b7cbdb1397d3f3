"""Summarise a rocprofv3 --pmc run (csv output): per kernel, dispatches and the
average of each counter per dispatch.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived metrics).  On gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming
read (MI355X_MICROARCH.md, HBM section), so `--gfx950-fetch-x2` doubles it:
the decode kernels read weights and K/V rows with 16-B loads.

Usage: python tools/pmc_summary.py DIR [kernel-substring] [--json OUT] [--gfx950-fetch-x2]
"""
import csv
import glob
import json
import sys


def load(path):
    files = glob.glob(path + "/**/*counter_collection.csv", recursive=True)
    agg = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = (r["Kernel_Name"], r["Counter_Name"])
                a = agg.setdefault(k, {})
                # one row per (dispatch, counter) once summed over dimensions
                d = r.get("Dispatch_Id") or r.get("Correlation_Id")
                a[d] = a.get(d, 0.0) + float(r["Counter_Value"])
    return agg


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_json = None
    if "--json" in sys.argv:
        out_json = sys.argv[sys.argv.index("--json") + 1]
        args = [a for a in args if a != out_json]
    x2 = "--gfx950-fetch-x2" in sys.argv
    path = args[0]
    filt = args[1] if len(args) > 1 else None
    agg = load(path)
    res = {}
    for (kn, cn), per in sorted(agg.items()):
        if filt and filt not in kn:
            continue
        vals = list(per.values())
        avg = sum(vals) / len(vals)
        if x2 and cn == "FETCH_SIZE":
            avg *= 2
        res.setdefault(kn, {})[cn] = {"dispatches": len(vals), "avg_per_dispatch": avg}
        print(f"{kn[:90]:90s} {cn:14s} n={len(vals):6d} avg={avg:.6g}")
    if out_json:
        with open(out_json, "w") as fh:
            json.dump({"source": path, "fetch_x2": x2, "kernels": res}, fh, indent=1)


if __name__ == "__main__":
    main()
