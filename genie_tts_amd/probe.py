"""Roofline of the dominant kernel, from the engine's live in-loop timing.

The dominant kernel is the persistent decode `k_decode_persist1`
(t2s_persist1.hip): ONE launch per utterance that runs every decode step.  Its
algorithmic bytes (per sequence per step): the fp16 weights read
once, W16 = 24 layers x (1536+512+2048+2048) x 512 x 2 B + the 1025x512 fp16
logits head = 152,044,544 B, plus the fp32 K/V cache rows read, 98,304 B per
cached position (24 layers x K,V x 512 x 4 B), plus the new row written,
98,304 B.  Summed over the launch's steps (key count N0 + s at step s).
The duration is the launch's own dispatch-packet start/stop events
(hipExtLaunchKernelGGL), averaged over the timed utterances.
"""
from __future__ import annotations

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


W16 = 24 * (1536 + 512 + 2048 + 2048) * 512 * 2 + 1025 * 512 * 2   # 152,044,544
KV_ROW = 24 * 2 * 512 * 4                                         # 98,304


def persist_algorithmic_bytes(n0: int, steps: int, B: int = 1) -> int:
    """Bytes one persistent launch must move: per step W16 once + each sequence's
    K/V rows read (n0 + s of them) and one row written."""
    return sum(W16 + B * (KV_ROW * (n0 + s) + KV_ROW) for s in range(steps))


# The translation unit k_decode_persist1 is compiled from: its HBM traffic depends on
# these files only, so a PMC count stays valid while other kernels change.
DECODE_TU = ("t2s_persist1.hip", "common.h", "kernels.h", "sampler.h", "persist.h")


def kernel_source_sha() -> str:
    """sha256 (16 hex) over the decode kernel's translation unit (DECODE_TU):
    identifies the kernel build a PMC measurement belongs to."""
    import hashlib
    import os
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    h = hashlib.sha256()
    for f in DECODE_TU:
        h.update(f.encode())
        h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel_sub: str):
    """HBM bytes per launch of the named kernel from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench).  None when
    there is none, or when it was measured on other kernel sources than the
    ones built here (its csrc_sha differs): a stale count is not reported."""
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    sha = kernel_source_sha()
    for k, v in d.get("kernels", {}).items():
        if kernel_sub in k:
            if d.get("csrc_sha") != sha:
                return None, f"stale: {d.get('source')} measured csrc {d.get('csrc_sha')}, built {sha}"
            return float(v["traffic_bytes"]), f"{d.get('source')}, csrc {sha}: {k}"
    return None, None


def persist_roofline(eng, n0: int, steps: int, B: int = 1):
    us, n = eng.kernel_timing()
    if n <= 0 or us <= 0:
        return {"error": f"no live kernel samples (hipEventElapsedTime error {-n})"}
    bytes_ = persist_algorithmic_bytes(n0, steps, B)
    achieved = bytes_ / (us * 1e-6) / 1e9
    traffic, tsrc = pmc_traffic("k_decode_persist")
    return {
        "kernel": "k_decode_persist (whole decode loop, %d steps, N0=%d, B=%d)" % (steps, n0, B),
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "traffic_source": tsrc,
        "algorithmic_bytes_per_launch": bytes_,
        "avg_launch_us": us,
        "samples": n,
    }


# ------------------------------------------------------------------ composite
# roofline.achieved of the whole utterance = sum over phases of the
# phase's minimum time on its own bound, over the measured time.
#   decode : algorithmic bytes (above) / HBM peak
#   prefill: 2 N0 x 24 x 3,145,728 (q/k/v, out, FFN1, FFN2 weights) + 4 N0^2 x 512 x 24
#            (dense scores and P.V) FLOP
#   vits   : 135.5 GFLOP (V2) / 298 GFLOP (V2ProPlus) per 80 tokens, linear in the
#            token count (the generator, 96 % of it, is linear in G)
# Two compute ceilings, both reported:
#   f32       : the FP32 matrix peak (the reference computes in fp32);
#   split_f16 : the precision the kernels actually run at -- the f16 MFMA (2.5 PF dense)
#               divided by the MFMAs each product costs: fp16 weights x (hi, lo) activation
#               = 2 (k_gemm_x3, k_conv_h; the prefill's attention and VITS' few f32-MFMA
#               convs are priced at this rate too, a lower bound on their time).
F32_PEAK_TFS = 157.3    # MI355X_MICROARCH.md: FP32 matrix peak
F16_PEAK_TFS = 2500.0   # MI355X_MICROARCH.md: BF16/FP16 MFMA, dense
SPLIT_F16_TFS = F16_PEAK_TFS / 2   # 2 MFMAs per product (activation hi + lo)
VITS_FLOP_PER_TOKEN = {"v2": 135.5e9 / 80, "v2ProPlus": 298.0e9 / 80}


def prefill_flop(n0: int) -> float:
    return 2.0 * n0 * 24 * 3145728 + 4.0 * n0 * n0 * 512 * 24


def batch_decode_bytes(n0s, steps) -> int:
    """Algorithmic bytes of a ragged batched decode: per loop step the fp16 weights
    once + each still-active sequence's K/V rows read and its new row written."""
    total = 0
    for s in range(max(steps)):
        act = [n0 for n0, st in zip(n0s, steps) if s < st]
        total += W16 + sum(KV_ROW * (n0 + s + 1) for n0 in act)
    return total


def composite_roofline(ms_total: float, n0s, steps, tokens, version: str = "v2", phase_ms=None):
    """Sum of per-phase minimum times / measured time for one job (ms_total), with the
    compute phases priced at the FP32 peak (frac) and at the split-fp16 MFMA ceiling
    the kernels run on (frac_split_f16)."""
    t_dec = batch_decode_bytes(n0s, steps) / (HBM_PEAK_GBS * 1e9) * 1e3
    f_pre = sum(prefill_flop(n0) for n0 in n0s)
    f_voc = sum(VITS_FLOP_PER_TOKEN[version] * g for g in tokens)
    t_pre, t_voc = f_pre / (F32_PEAK_TFS * 1e12) * 1e3, f_voc / (F32_PEAK_TFS * 1e12) * 1e3
    h_pre, h_voc = f_pre / (SPLIT_F16_TFS * 1e12) * 1e3, f_voc / (SPLIT_F16_TFS * 1e12) * 1e3
    out = {"t_min_ms": {"decode_hbm": t_dec, "prefill_f32": t_pre, "vits_f32": t_voc,
                        "prefill_split_f16": h_pre, "vits_split_f16": h_voc},
           "t_measured_ms": ms_total, "frac": (t_dec + t_pre + t_voc) / ms_total,
           "frac_split_f16": (t_dec + h_pre + h_voc) / ms_total,
           "peaks": {"hbm_GBs": HBM_PEAK_GBS, "f32_TFs": F32_PEAK_TFS, "split_f16_TFs": SPLIT_F16_TFS}}
    if phase_ms:
        mins = {"decode": t_dec, "prefill": t_pre, "vits": t_voc}
        mins_h = {"decode": t_dec, "prefill": h_pre, "vits": h_voc}
        out["phase_frac"] = {k: mins[k] / v for k, v in phase_ms.items() if k in mins and v > 0}
        out["phase_frac_split_f16"] = {k: mins_h[k] / v for k, v in phase_ms.items() if k in mins_h and v > 0}
    return out
