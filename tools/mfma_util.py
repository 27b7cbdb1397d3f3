"""MFMA utilisation per kernel from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (csv output).

util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / 8): the busy cycles summed
over every SIMD against the cycles the chip was active for the dispatch (GRBM_GUI_ACTIVE
sums the 8 XCDs, MI355X_MICROARCH.md), i.e. the fraction of the f16/bf16 MFMA peak the
kernel's MFMA pipes were issuing.  A split-fp16 product (2 MFMAs) or a hi/lo-weight one
(3) counts every MFMA, so the useful-FLOP fraction is util / 2 or util / 3.

Usage: python tools/mfma_util.py DIR [--simds 1024]
"""
import sys

sys.path.insert(0, "tools")
from pmc_summary import load  # noqa: E402


def main():
    path = sys.argv[1]
    simds = int(sys.argv[sys.argv.index("--simds") + 1]) if "--simds" in sys.argv else 1024
    agg = load(path)
    per = {}
    for (kn, cn), d in agg.items():
        per.setdefault(kn, {})[cn] = d
    rows = []
    for kn, c in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        m, g = c["SQ_VALU_MFMA_BUSY_CYCLES"], c["GRBM_GUI_ACTIVE"]
        ids = [k for k in m if k in g]
        mb = sum(m[k] for k in ids)
        ga = sum(g[k] for k in ids)
        if ga <= 0:
            continue
        rows.append((mb / (simds * ga / 8.0), len(ids), mb / max(1, len(ids)), ga / 8.0 / max(1, len(ids)), kn))
    rows.sort(key=lambda r: -r[2] * r[1])
    print(f"{'mfma_util':>9s} {'n':>6s} {'busy_cyc/disp':>14s} {'active_cyc/disp':>15s}  kernel")
    for u, n, mb, ga, kn in rows:
        print(f"{u:9.4f} {n:6d} {mb:14.4g} {ga:15.4g}  {kn[:100]}")


if __name__ == "__main__":
    main()
