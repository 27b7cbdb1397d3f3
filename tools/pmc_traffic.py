"""Combine the FETCH_SIZE / WRITE_SIZE passes of one GPU round (tools/gpu_round.sh
pmc step) into profiles/pmc_traffic.json, read by bench.py for roofline.traffic.

traffic per launch = 2 x FETCH_SIZE (gfx950 half-count correction for 16-B
streaming reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, in bytes (KB = 1024).
Usage: python tools/pmc_traffic.py TAG [kernel-substring]
"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
from genie_tts_amd.probe import kernel_source_sha  # noqa: E402

tag = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_decode_persist"
f = json.load(open(f"gpurun_out/{tag}_pmc_FETCH_SIZE.json"))["kernels"]
w = json.load(open(f"gpurun_out/{tag}_pmc_WRITE_SIZE.json"))["kernels"]
out = {}
for k, v in f.items():
    if sub not in k:
        continue
    fk = v["FETCH_SIZE"]["avg_per_dispatch"]          # already x2 (pmc_summary --gfx950-fetch-x2)
    wk = w.get(k, {}).get("WRITE_SIZE", {}).get("avg_per_dispatch", 0.0)
    out[k] = {"fetch_bytes_x2": fk * 1024, "write_bytes": wk * 1024, "traffic_bytes": (fk + wk) * 1024,
              "dispatches": v["FETCH_SIZE"]["dispatches"]}
json.dump({"round": tag, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py ({tag})",
           "csrc_sha": kernel_source_sha(), "kernels": out}, open("profiles/pmc_traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
