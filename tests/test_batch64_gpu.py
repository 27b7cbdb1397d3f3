"""configs[2] on the GPU: 64 mixed-length JP sentences in ONE batched decode
(S~U[30,60], forced G~U[50,110]; genie_tts_amd.workloads.batch64) through the
C ABI (gsv_t2s_generate with per-utterance force_steps), against the oracle's
tokens in tests/golden/t2s_batch64.npz (tests/golden/make_batch64.py; pinned
to oracle/restate.py by tests/test_batch64_oracle.py):

  greedy   per-utterance token ids bit-exact (the north_star's bar);
  top-k 5  per-utterance token ids identical to the oracle loop fed the same
           Philox N(0,1) noise (tests/philox.py) -- the sampled formula
           argmax(softmax(top-k(penalised logits)) / q) of
           t2s_stage_decoder_fp32.onnx#1775-1806.
"""
import os

import numpy as np
import pytest

from tests.common import character

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "t2s_batch64.npz")


@pytest.fixture(scope="module")
def eng():
    from genie_tts_amd.engine import Engine
    w = character("v2")
    e = Engine({"t2s_encoder": w["t2s_encoder"], "t2s": w["t2s"]}, "v2")
    yield e
    e.close()


def _utts(wl):
    ref = wl.reference
    return [(ref.ref_seq, it.text_seq, None, None, ref.ssl.reshape(768, -1), it.force_steps) for it in wl.items]


@pytest.mark.parametrize("mode", ["greedy", "topk"])
def test_batch64_matches_oracle(eng, mode):
    from genie_tts_amd import workloads
    from genie_tts_amd.engine import make_sampler
    g = np.load(GOLD)
    wl = workloads.batch64()
    assert [it.tokens for it in wl.items] == g["G"].tolist()
    sp = make_sampler(top_k=int(g["top_k"]) if mode == "topk" else 15, greedy=(mode == "greedy"),
                      seed=int(g["seed"]))
    out = eng.t2s_generate(_utts(wl), sp)
    bad = []
    for b, tok in enumerate(out):
        ref = g[mode][b, :g[mode + "_len"][b]].astype(np.int64)
        if tok.tolist() != ref.tolist():
            n = min(tok.size, ref.size)
            i = next((j for j in range(n) if tok[j] != ref[j]), n)
            bad.append((b, i, tok[max(0, i - 2):i + 3].tolist(), ref[max(0, i - 2):i + 3].tolist()))
    assert not bad, f"{mode}: (utterance, first differing token, engine, oracle) {bad}"


def test_batch64_ragged_lengths(eng):
    """Each utterance stops at its own forced length; finished rows are skipped
    by the rest of the batch (ragged KV), so lengths equal G exactly."""
    from genie_tts_amd import workloads
    from genie_tts_amd.engine import make_sampler
    wl = workloads.batch64(16, tag="b64r")
    out = eng.t2s_generate(_utts(wl), make_sampler())
    assert [o.size for o in out] == [it.tokens for it in wl.items]


def test_packed_prefill_attention_matches_per_sequence_prefill(eng):
    """The packed prefill against the per-sequence prefill: the layer-23 K/V rows that every
    earlier layer's attention feeds, for 8 ragged utterances of batch64.  Since r05 the
    packed prefill's attention runs the f32 kernels the per-sequence prefill runs (the
    split-fp16 MFMA kernel k_attn_mfma is opt-in, GENIE_ATTN_MFMA=1: it flipped a near-tie
    token against the sentence alone, test_persistm_gpu.py), so the rows are bit-identical;
    with the MFMA kernel the bar is max |diff| <= 1e-4 x max |value|.  The packed side runs
    k_attn_mf32 (the f32 MFMA, 128-row tiles), the per-sequence side k_attn_flash itself
    (option attn_mf32 = 0)."""
    import os
    from genie_tts_amd import workloads
    from genie_tts_amd.engine import make_sampler
    wl = workloads.batch64()
    utts = [u[:5] + (1,) for u in _utts(wl)[:8]]   # one loop step: the prefill's K/V, then the cache
    sp = make_sampler(top_k=5, greedy=True)
    kv = {}
    try:
        for packed in (1, 0):
            eng.set_option("packed", packed)
            eng.set_option("attn_mf32", packed)   # per-sequence side on k_attn_flash itself
            eng.t2s_generate(utts, sp)
            kv[packed] = [[t.cpu().numpy() for t in eng.t2s_read_kv(23, seq=b)] for b in range(len(utts))]
    finally:
        eng.set_option("packed", 1)
        eng.set_option("attn_mf32", 1)
    for b in range(len(utts)):
        for a, r in zip(kv[1][b], kv[0][b]):
            assert a.shape == r.shape and a.shape[0] > 128
            err = float(np.abs(a - r).max())
            if os.environ.get("GENIE_ATTN_MFMA", "0") not in ("", "0"):
                assert err <= 1e-4 * float(np.abs(r).max()), (b, err)
            else:
                assert err == 0.0, (b, err)


def test_single_prefill_attention_mf32_matches_flash(eng):
    """One sentence's prefill with its attention on k_attn_mf32 (32-row single-wave
    blocks; GENIE_PREFILL_MF32=1, else this compares k_attn_flash with itself) and on
    k_attn_flash (option attn_mf32 = 0): layer-0 and layer-23 K/V bit-identical, and the
    same tokens over 20 steps.  The f32 MFMA computes each element as a sequential fma
    chain (tools/mfma_f32_probe.hip), so the kernels' per-row arithmetic is the same;
    r05m ran it with GENIE_PREFILL_MF32=1."""
    from genie_tts_amd import workloads
    from genie_tts_amd.engine import make_sampler
    wl = workloads.batch64(4, tag="mf32")
    sp = make_sampler(top_k=5, greedy=True)
    for u in _utts(wl):
        u = u[:5] + (20,)
        got = {}
        try:
            for mf in (1, 0):
                eng.set_option("attn_mf32", mf)
                toks = eng.t2s_generate([u], sp)[0]
                got[mf] = (toks.tolist(), [[t.cpu().numpy() for t in eng.t2s_read_kv(l, seq=0)] for l in (0, 23)])
        finally:
            eng.set_option("attn_mf32", 1)
        assert got[1][0] == got[0][0]
        for la, lr in zip(got[1][1], got[0][1]):
            for a, r in zip(la, lr):
                assert a.shape == r.shape and np.array_equal(a, r)
