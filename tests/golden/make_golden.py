#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run in the build container only).

Each fixture is produced by executing the reference's own ONNX graph templates
(`/root/reference/src/genie_tts/Data/{v2,v2ProPlus}/Models/*.onnx`) with the
numpy executor in oracle/onnx_interp.py -- i.e. the exact op graph Genie hands
to onnxruntime (`g/Core/Inference.py:76,88,102,47,55`) -- on synthetic
fp16-valued weights (genie_tts_amd.synth, seed 0x6E1E; the weights are not
stored, only a fingerprint that pins the generator) and seeded inputs.
`RandomNormalLike` substitutions: T2S := 1 (greedy), VITS := 0 or a stored eps.

Fixtures hold inputs and outputs only (data), never reference source.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from genie_tts_amd import synth, weights as W  # noqa: E402
from oracle import graphs as G  # noqa: E402


def fingerprint(w):
    keys = sorted(w)
    return np.array([float(np.abs(np.asarray(w[k], np.float64)).sum()) for k in keys], np.float64)


def t2s_case(name, R, S, H, steps, w_enc, w_t2s, kv_layers=(0, 23), force_eos=False):
    t0 = time.time()
    ref = synth.synth_phones(R, "gold-r" + name)
    txt = synth.synth_phones(S, "gold-t" + name)
    rb = np.zeros((R, 1024), np.float32)
    tb = np.zeros((S, 1024), np.float32)
    ssl = synth.synth_ssl(H, "gold-s" + name)
    x, prompts = G.t2s_encoder(w_enc, ref, txt, rb, tb, ssl)
    g = G.graph("v2/Models/t2s_first_stage_decoder_fp32.onnx")
    out = G.t2s_first_stage(w_t2s, x, prompts)
    y, y_emb, kv = out[0], out[1], out[2:]
    from oracle.onnx_interp import Interpreter
    it = Interpreter(g, {k: np.asarray(v, np.float32) for k, v in w_t2s.items()}, random_normal=G.ones_like)
    prefill_logits = it.run(dict(x=x, prompts=prompts), ["/Gather_3_output_0"])[0]
    step_logits, step_tokens, stops = [], [], []
    cur = (y, y_emb, kv)
    gs = G.graph("v2/Models/t2s_stage_decoder_fp32.onnx")
    names = [i[0] for i in gs.inputs]
    its = Interpreter(gs, {k: np.asarray(v, np.float32) for k, v in w_t2s.items()}, random_normal=G.ones_like)
    idx = 0
    for idx in range(steps):
        feeds = {n: v for n, v in zip(names, [cur[0], cur[1], *cur[2]])}
        res = its.run(feeds, [o[0] for o in gs.outputs] + ["/Gather_1_output_0"])
        yy, ye, stop = res[0], res[1], res[2]
        kvn = res[3:-1]
        step_logits.append(res[-1])
        step_tokens.append(int(yy[0, -1]))
        stops.append(bool(stop))
        cur = (yy, ye, kvn)
        if force_eos and stop:
            break
    yfin = cur[0].copy()
    yfin[0, -1] = 0
    sem = np.expand_dims(yfin[:, -idx:], axis=0)
    sem = G.eos_filter(sem)
    d = dict(ref_seq=ref, text_seq=txt, ssl=ssl, x=x, prompts=prompts, y_prefill=y,
             prefill_logits=prefill_logits, step_logits=np.stack(step_logits),
             step_tokens=np.array(step_tokens, np.int64), stops=np.array(stops),
             pred_semantic=sem, loop_idx=np.array(idx))
    for l in kv_layers:
        d[f"kv_k{l}"] = kv[2 * l][:, 0]
        d[f"kv_v{l}"] = kv[2 * l + 1][:, 0]
    print(f"  t2s {name}: {time.time() - t0:.1f}s steps={len(step_tokens)} stop={stops[-1]}", flush=True)
    return d


VITS_FETCH = {
    "v2": {"ge": "/vq_model/ref_enc/Unsqueeze_6_output_0"},
    "v2ProPlus": {},
}


def vits_case(ver, Gn, S, w):
    t0 = time.time()
    txt = synth.synth_phones(S, f"gold-vt{ver}")
    sem = (synth.rng_for(f"gold-sem{ver}").integers(0, 1024, size=Gn)).astype(np.int64).reshape(1, 1, Gn)
    eps = synth.rng_for(f"gold-eps{ver}").standard_normal((1, 192, 2 * Gn)).astype(np.float32)
    if ver == "v2":
        kw = dict(ref_audio=synth.synth_ref_audio(32000 * 2 + 777, "gold"))
    else:
        kw = dict(ge=synth.synth_ge(1024, "gold"), ge_advanced=synth.synth_ge(512, "gold-adv"))
    fetch = ["audio", "/vq_model/enc_p/Split_output_0", "/vq_model/enc_p/Split_output_1"] + \
        list(VITS_FETCH[ver].values())
    zero = G.vits(ver, w, txt, sem, noise=G.zeros_like, fetch=fetch, **kw)
    noisy = G.vits(ver, w, txt, sem, noise=lambda x, a: eps, fetch=["audio"], **kw)[0]
    d = dict(text_seq=txt, pred_semantic=sem, eps=eps, audio_zero=zero[0], audio_eps=noisy,
             m_p=zero[1], logs_p=zero[2], **{k: v for k, v in kw.items()})
    for i, k in enumerate(VITS_FETCH[ver]):
        d[k] = zero[3 + i]
    print(f"  vits {ver}: {time.time() - t0:.1f}s", flush=True)
    return d


def main():
    assert G.available(), "reference graph templates not found"
    out = HERE
    # PE div_term constant exactly as stored in the graphs (stage#21)
    g = G.graph("v2/Models/t2s_stage_decoder_fp32.onnx")
    div = next(n for n in g.nodes if n.outputs[0] == "/ar_audio_position/Constant_1_output_0")
    np.save(os.path.join(out, "pe_div_term.npy"), div.attrs["value"].numpy().astype(np.float32))

    w_enc = synth.synth_weights(W.t2s_encoder_spec(), fp16=False)
    w_t2s = synth.synth_weights(W.t2s_spec())
    np.savez_compressed(os.path.join(out, "weights_fingerprint.npz"),
                        t2s_encoder=fingerprint(w_enc), t2s=fingerprint(w_t2s),
                        vits_v2=fingerprint(synth.synth_weights(W.vits_spec("v2"))),
                        vits_v2pp=fingerprint(synth.synth_weights(W.vits_spec("v2ProPlus"))),
                        prompt_encoder=fingerprint(synth.synth_weights(W.prompt_encoder_spec())))
    np.savez_compressed(os.path.join(out, "t2s_small.npz"), **t2s_case("small", 12, 10, 41, 8, w_enc, w_t2s))
    np.savez_compressed(os.path.join(out, "t2s_nominal.npz"),
                        **t2s_case("nominal", 48, 45, 264, 40, w_enc, w_t2s, kv_layers=(0,)))
    # forced EOS: layer-23 norm2 ~ 0, bias b, EOS row = 10 b
    w_eos = dict(w_t2s)
    b = np.asarray(w_t2s["transformer_encoder.layers.23.norm2.bias"], np.float32)
    w_eos["transformer_encoder.layers.23.norm2.weight"] = np.full(512, 1e-3, np.float16)
    pred = np.asarray(w_t2s["ar_predict_layer.weight"], np.float32).copy()
    pred[1024] = 10.0 * b
    w_eos["ar_predict_layer.weight"] = pred.astype(np.float16)
    np.savez_compressed(os.path.join(out, "t2s_eos.npz"),
                        **t2s_case("eos", 12, 10, 41, 5, w_enc, w_eos, kv_layers=(), force_eos=True))
    for ver in ("v2", "v2ProPlus"):
        w = synth.synth_weights(W.vits_spec(ver))
        np.savez_compressed(os.path.join(out, f"vits_{ver}.npz"), **vits_case(ver, 8, 10, w))
    # prompt encoder (V2ProPlus)
    wp = synth.synth_weights(W.prompt_encoder_spec())
    ra = synth.synth_ref_audio(32000 * 3, "gold-pe")
    sv = synth.rng_for("gold-sv").standard_normal((1, 20480)).astype(np.float32)
    ge, ga = G.prompt_encoder(wp, ra, sv)
    np.savez_compressed(os.path.join(out, "prompt_encoder.npz"), ref_audio=ra, sv_emb=sv, ge=ge, ge_advanced=ga)
    print("done")


if __name__ == "__main__":
    main()
