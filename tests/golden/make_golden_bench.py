#!/usr/bin/env python3
"""Golden fixtures at the bench workload's sizes (run in the build container only).

Like make_golden.py, every output comes from executing the reference's own ONNX
graph templates with the numpy executor (oracle/onnx_interp.py) on the synthetic
fp16-valued weights (genie_tts_amd.synth, seed 0x6E1E).  The noise sources are
pinned to the engine's own Philox streams (tests/philox.py) instead of the
constant substitutions, so the SAMPLED formula of the graphs is pinned too:

  t2s_nominal81.npz   configs[1] nominal utterance (R=48, S=45, H=264; the inputs
                      of t2s_nominal.npz), 81 loop steps, greedy
                      (RandomNormalLike := 1, t2s_stage_decoder_fp32.onnx#1799)
  t2s_sampled81.npz   the same inputs, top-k 15 sampled: RandomNormalLike := the
                      engine's Philox N(0,1) q (first stage: Philox step 0,
                      t2s_first_stage_decoder_fp32.onnx#1813; loop step i: step
                      i + 1; batch slot 0; seed 1234)
  vits_{ver}_g80.npz  G=80, S=45 (the bench's 102,400 samples): RandomNormalLike
                      := 0 and := the engine's Philox eps of z_p (seed 77),
                      vits_fp32.onnx(v2)#6490 / (v2pp)#6225

Fixtures hold inputs and outputs only (data).  Runtime: a few minutes on 8 cores.
"""
from __future__ import annotations

import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

STEPS = 81
T2S_SEED = 1234
VITS_SEED = 77


def t2s_run(sampled: bool):
    from genie_tts_amd import synth, weights as W
    from oracle import graphs as G
    from tests.philox import sampler_noise

    t0 = time.time()
    nom = dict(np.load(os.path.join(HERE, "t2s_nominal.npz"), allow_pickle=False))
    w_enc = synth.synth_weights(W.t2s_encoder_spec(), fp16=False)
    w_t2s = synth.synth_weights(W.t2s_spec())
    R, S = nom["ref_seq"].shape[1], nom["text_seq"].shape[1]
    state = {"step": 0}

    def noise(x, a):
        if not sampled:
            return np.ones_like(x, dtype=np.float32)
        assert x.shape[-1] == 1025, x.shape
        return sampler_noise(1025, state["step"], 0, T2S_SEED).reshape(x.shape)

    x, prompts = G.t2s_encoder(w_enc, nom["ref_seq"], nom["text_seq"], np.zeros((R, 1024), np.float32),
                               np.zeros((S, 1024), np.float32), nom["ssl"])
    assert np.array_equal(prompts, nom["prompts"])
    y, y_emb, *kv = G.t2s_first_stage(w_t2s, x, prompts, noise)
    y0 = y.copy()
    tokens, stops = [], []
    for i in range(STEPS):
        state["step"] = i + 1
        y, y_emb, stop, *kv = G.t2s_stage(w_t2s, y, y_emb, kv, noise)
        tokens.append(int(y[0, -1]))
        stops.append(bool(stop))
    yfin = y.copy()
    yfin[0, -1] = 0
    sem = G.eos_filter(np.expand_dims(yfin[:, -(STEPS - 1):], axis=0))
    print(f"  t2s {'sampled' if sampled else 'greedy'}: {time.time() - t0:.1f}s", flush=True)
    return dict(y_prefill=y0, step_tokens=np.array(tokens, np.int64), stops=np.array(stops),
                pred_semantic=sem, seed=np.array(T2S_SEED if sampled else 0, np.int64),
                top_k=np.array(15, np.int64))


def vits_run(ver: str):
    from genie_tts_amd import synth, weights as W
    from oracle import graphs as G
    from tests.philox import vits_noise

    t0 = time.time()
    w = synth.synth_weights(W.vits_spec(ver))
    Gn, S = 80, 45
    txt = synth.synth_phones(S, f"gold80-vt{ver}")
    sem = synth.rng_for(f"gold80-sem{ver}").integers(0, 1024, size=Gn).astype(np.int64).reshape(1, 1, Gn)
    if ver == "v2":
        kw = dict(ref_audio=synth.synth_ref_audio(169600, "gold80"))
    else:
        kw = dict(ge=synth.synth_ge(1024, "gold80"), ge_advanced=synth.synth_ge(512, "gold80-adv"))
    zero = G.vits(ver, w, txt, sem, noise=G.zeros_like, fetch=["audio"], **kw)[0]
    noisy = G.vits(ver, w, txt, sem, noise=lambda x, a: vits_noise(x.size, VITS_SEED).reshape(x.shape),
                   fetch=["audio"], **kw)[0]
    print(f"  vits {ver} G=80: {time.time() - t0:.1f}s", flush=True)
    return dict(text_seq=txt, pred_semantic=sem, audio_zero=zero.astype(np.float32),
                audio_philox=noisy.astype(np.float32), noise_seed=np.array(VITS_SEED, np.int64), **kw)


def main():
    from oracle import graphs as G
    assert G.available(), "reference graph templates not found"
    jobs = {"t2s_nominal81.npz": (t2s_run, False), "t2s_sampled81.npz": (t2s_run, True),
            "vits_v2_g80.npz": (vits_run, "v2"), "vits_v2ProPlus_g80.npz": (vits_run, "v2ProPlus")}
    only = sys.argv[1:]
    with ProcessPoolExecutor(max_workers=4) as ex:
        futs = {name: ex.submit(fn, arg) for name, (fn, arg) in jobs.items() if not only or name in only}
        for name, f in futs.items():
            np.savez_compressed(os.path.join(HERE, name), **f.result())
            print("wrote", name, flush=True)


if __name__ == "__main__":
    main()
