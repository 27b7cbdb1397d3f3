#!/usr/bin/env python3
"""Benchmark: GPT-SoVITS inference (Genie hot path) on MI355X.

Metric (BASELINE.json): real-time factor + utterances/sec, 20-char JP, V2 speaker.
Workload (configs[1]): one V2 utterance through the whole path -- T2S encoder,
prefill, greedy decode (forced to 81 loop steps -> 80 semantic tokens, since
random weights never emit EOS), VITS (ref STFT + MelStyleEncoder, TextEncoder,
flow, HiFi-GAN) -> 102,400 samples = 3.2 s of 32 kHz audio.  Nominal shapes
(SURVEY §8): reference phones R=48, target phones S=45, HuBERT frames H=264
(P=132 prompts), reference audio 5.3 s.  Synthetic weights/inputs (no
checkpoints offline).  A "step" = one utterance; inputs are resident in HBM.

Multi-GPU: one process per GPU (torchrun), independent replicas, no
collective on the data path; barrier + max-over-ranks timing; value = all
utterances / max time (weak scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "real-time factor + utterances/sec, 20-char JP, V2 speaker, 1/2/4/8 MI355X"
R_PH, S_PH, H_SSL = 48, 45, 264
FORCE_STEPS = 81                 # loop steps -> 80 kept tokens (Inference.py:108-109 trim)
REF_AUDIO_S = 5.3
SR = 32000
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
F32_MFMA_PEAK_TFS = 157.3        # MI355X_MICROARCH.md: FP32 matrix (= vector) peak


def build_inputs():
    from genie_tts_amd import synth
    ref = synth.synth_phones(R_PH, "bench-ref")
    txt = synth.synth_phones(S_PH, "bench-text")
    rb = np.zeros((R_PH, 1024), np.float32)          # JP: BERT features are zeros
    tb = np.zeros((S_PH, 1024), np.float32)
    ssl = synth.synth_ssl(H_SSL, "bench")
    audio = synth.synth_ref_audio(int(REF_AUDIO_S * SR), "bench")
    return ref, txt, rb, tb, ssl, audio


def cpu_baseline(inputs, threads: int):
    """Oracle restatement of Genie's ONNX-CPU path on the host cores (torch fp32)."""
    import torch
    from genie_tts_amd import synth
    from oracle import restate as R
    torch.set_num_threads(threads)
    w = synth.synthetic_character("v2")
    m = R.T2SModel(w["t2s"])
    vm = R.VitsModel(w["vits"], "v2")
    ref, txt, rb, tb, ssl, audio = inputs
    t0 = time.perf_counter()
    sem, _, _ = R.t2s_generate(w["t2s_encoder"], m, ref, rb, txt, tb, ssl, force_steps=FORCE_STEPS)
    wav = vm(txt, sem, ref_audio=audio)
    dt = time.perf_counter() - t0
    return dt, int(wav.numel())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from genie_tts_amd import synth
    from genie_tts_amd.engine import Engine, make_sampler
    w = synth.synthetic_character("v2")
    eng = Engine(w, "v2", device=local if world > 1 else 0)
    inputs = build_inputs()
    ref, txt, rb, tb, ssl, audio = inputs
    dev = torch.device("cuda", local if world > 1 else 0)
    # inputs resident in HBM before the timed region (warmup triggers the graph captures)
    d_ref = torch.as_tensor(ref.reshape(-1), device=dev)
    d_txt = torch.as_tensor(txt.reshape(-1), device=dev)
    d_ssl = torch.as_tensor(ssl.reshape(768, -1), device=dev)
    d_audio = torch.as_tensor(audio.reshape(-1), device=dev)
    sp = make_sampler(force_steps=FORCE_STEPS)
    eng.set_option("persist", 1)  # whole decode loop as one launch (t2s_persist.hip)
    eng.set_timing(True)          # phase events + live dominant-kernel event pair

    def one_utterance():
        sem = eng.t2s_generate([(d_ref, d_txt, None, None, d_ssl)], sp)[0]
        wav = eng.vits_decode(d_txt, sem, ref_audio=d_audio)
        return sem, wav

    for _ in range(args.warmup):
        sem, wav = one_utterance()
    torch.cuda.synchronize()
    eng.set_timing(True)          # reset live-kernel samples: only the timed region counts
    n_tokens = int(sem.size)
    n_samples = int(wav.numel())
    audio_s = n_samples / SR

    phase_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_utterance()
        phase_ms.append(eng.timing())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_per_step = dt / args.steps * 1e3
    utt_s = world * args.steps / dt
    rtf = (dt / args.steps) / audio_s

    from genie_tts_amd.probe import persist_roofline
    roofline = persist_roofline(eng, n0=R_PH + S_PH + H_SSL // 2, steps=FORCE_STEPS, B=1)

    out = {
        "metric": METRIC,
        "value": utt_s,
        "unit": "utt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (fp16-valued weights)",
        "data": "synthetic (seeded inputs, synthetic fp16-valued weights; no checkpoints offline)",
        "rtf": rtf,
        "x_realtime": 1.0 / rtf,
        "audio_s_per_utt": audio_s,
        "tokens_per_utt": n_tokens,
        "config": {"workload": "configs[1]: V2 speaker, single utterance, greedy, 1 utt per replica",
                   "ref_phones": R_PH, "text_phones": S_PH, "ssl_frames": H_SSL,
                   "loop_steps": FORCE_STEPS, "semantic_tokens": n_tokens,
                   "samples": n_samples, "parallelism": f"replicas x{world}"},
        "roofline": roofline,
    }
    if phase_ms:
        pm = np.mean(np.asarray(phase_ms), axis=0)
        out["phase_ms"] = {"encode": float(pm[0]), "prefill": float(pm[1]), "decode": float(pm[2]),
                           "vits": float(pm[3])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, len(os.sched_getaffinity(0)))
        cdt, cs = cpu_baseline(inputs, threads)
        model = ""
        try:
            with open("/proc/cpuinfo") as f:
                model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
        except Exception:
            pass
        out["cpu_baseline"] = {"value": 1.0 / cdt, "unit": "utt/s", "cores": threads, "kind": "port",
                               "sample": f"1 full utterance ({cs} samples) of the same workload, "
                                         f"oracle/restate.py torch-fp32 on {model}",
                               "rtf": cdt / (cs / SR)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
