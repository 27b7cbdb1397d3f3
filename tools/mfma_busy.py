"""MFMA-busy per phase from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run of bench.py.  SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipeline cycles summed over
SIMDs (32 per v_mfma_*_32x32x16 f16/bf16, MI355X_MICROARCH.md PMC units);
GRBM_GUI_ACTIVE counts GPU-active cycles summed over the 8 XCDs.  busy fraction =
MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs) = the share of the
chip's MFMA issue slots used while the kernels ran.
Usage: python tools/mfma_busy.py DIR [--json OUT]"""
import json
import sys

sys.path.insert(0, "tools")
from pmc_summary import load  # noqa: E402

PHASES = {
    "decode": ("k_decode_persist",),
    "prefill": ("k_gemm_x2", "k_attn_rows", "k_layernorm512_slabs"),
    "vits": ("k_conv_h", "k_conv1d", "k_conv_reduce", "k_mha", "k_ln_channels", "k_wn_gate", "k_gemm_nt",
             "k_time_mean", "k_flip", "k_glu", "k_noise", "k_cb_up2", "k_embed_ch", "k_flow", "k_stft"),
}


def main():
    path = sys.argv[1]
    agg = load(path)
    per = {}
    for (kn, cn), d in agg.items():
        e = per.setdefault(kn, {})
        e[cn] = sum(d.values())
        e["n"] = len(d)
    out = {"kernels": {}, "phases": {}}
    for kn, e in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
        busy, act = e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), e.get("GRBM_GUI_ACTIVE", 0.0)
        if act <= 0:
            continue
        frac = busy / (act / 8 * 1024)
        out["kernels"][kn] = {"dispatches": e["n"], "mfma_busy_cycles": busy, "gui_active": act, "busy_frac": frac}
    for ph, subs in PHASES.items():
        b = sum(v["mfma_busy_cycles"] for k, v in out["kernels"].items() if any(s in k for s in subs))
        a = sum(v["gui_active"] for k, v in out["kernels"].items() if any(s in k for s in subs))
        out["phases"][ph] = {"busy_frac": b / (a / 8 * 1024) if a else None, "mfma_busy_cycles": b, "gui_active": a}
    for ph, v in out["phases"].items():
        print(f"phase {ph:8s} MFMA busy {100 * (v['busy_frac'] or 0):6.2f} %")
    for kn, v in list(out["kernels"].items())[:20]:
        print(f"  {kn[:80]:80s} n={v['dispatches']:5d} busy {100 * v['busy_frac']:6.2f} %")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
