#!/usr/bin/env python3
"""Generate tests/golden/t2s_batch64.npz: the configs[2] workload (64 mixed-length
JP sentences, S~U[30,60], forced G~U[50,110]; genie_tts_amd.workloads.batch64)
through the CPU oracle (oracle/restate.py, itself pinned to the reference graph
templates by tests/test_oracle.py), in two sampler modes:

  greedy   RandomNormalLike := 1 (t2s_stage_decoder_fp32.onnx#1799) -> argmax
  top-k 5  argmax(p / q) with q = the engine's Philox N(0,1) stream
           (tests/philox.py): first-stage token (Philox step 0) and loop step
           i (Philox step i + 1), both keyed by the utterance's batch slot b.

Loop `Inference.py:95-106` with forced lengths, trim + EOS filter
`Inference.py:108-109, 41-44`.  Fixture = inputs' lengths + output token ids
(data only).  Runs ~1 min on 8 cores.
"""
from __future__ import annotations

import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SEED = 1234
TOP_K = 5


def oracle_tokens(b: int, greedy: bool, n: int = 64):
    """Trimmed tokens of utterance b of the batch64 workload (oracle/restate.py)."""
    import torch
    torch.set_num_threads(1)
    from genie_tts_amd import synth, workloads
    from oracle import restate as R
    from tests.philox import sampler_noise
    w = _char()
    wl = workloads.batch64(n)
    it, ref = wl.items[b], wl.reference
    q_fn = None
    cfg = R.SamplerCfg()
    if not greedy:
        cfg = R.SamplerCfg(top_k=TOP_K)
        q_fn = lambda idx: torch.from_numpy(sampler_noise(1025, idx + 1, b, SEED))   # idx -1: first stage
    m = _model()
    sem, _, _ = R.t2s_generate(w["t2s_encoder"], m, ref.ref_seq, ref.ref_bert, it.text_seq,
                               np.zeros((it.text_seq.shape[1], 1024), np.float32), ref.ssl, cfg,
                               force_steps=it.force_steps, q_fn=q_fn)
    return np.asarray(sem).reshape(-1)


_CACHE = {}


def _char():
    if "w" not in _CACHE:
        from genie_tts_amd import synth
        _CACHE["w"] = synth.synthetic_character("v2")
    return _CACHE["w"]


def _model():
    if "m" not in _CACHE:
        from oracle import restate as R
        _CACHE["m"] = R.T2SModel(_char()["t2s"])
    return _CACHE["m"]


def _job(args):
    b, greedy = args
    return b, greedy, oracle_tokens(b, greedy)


def main():
    from genie_tts_amd import workloads
    wl = workloads.batch64()
    n = len(wl.items)
    G = np.array([it.tokens for it in wl.items], np.int32)
    S = np.array([it.text_seq.shape[1] for it in wl.items], np.int32)
    out = {True: np.full((n, G.max()), -1, np.int16), False: np.full((n, G.max()), -1, np.int16)}
    lens = {True: np.zeros(n, np.int32), False: np.zeros(n, np.int32)}
    jobs = [(b, g) for g in (True, False) for b in range(n)]
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for b, g, tok in ex.map(_job, jobs):
            out[g][b, :tok.size] = tok
            lens[g][b] = tok.size
    np.savez_compressed(os.path.join(HERE, "t2s_batch64.npz"), S=S, G=G, seed=np.int64(SEED), top_k=np.int32(TOP_K),
                        greedy=out[True], greedy_len=lens[True], topk=out[False], topk_len=lens[False])
    print("greedy lens", lens[True].tolist())
    print("top-k lens", lens[False].tolist())


if __name__ == "__main__":
    main()
