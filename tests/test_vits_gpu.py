"""VITS parity on the GPU: HIP engine (C ABI) vs the CPU oracle restatement.

Bar (north_star): waveform RMS difference <= 1e-4 in fp32 on identical inputs
and noise.  Oracle = oracle/restate.py, pinned to the reference graphs by
tests/test_oracle.py and the golden fixtures.
"""
import numpy as np
import pytest

from genie_tts_amd import synth
from tests.common import character

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4


def _close(got, want, what=""):
    """A segmented-batch result (one generator pass over the whole batch,
    option seg_vocoder) vs the same utterance decoded alone: the batch's larger tiles
    order the MRF reductions differently, so they agree to fp32 rounding, not bit for bit."""
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape, what
    rel = float(np.sqrt(np.mean((got - want) ** 2)) / max(1e-12, np.sqrt(np.mean(want ** 2))))
    assert rel <= 1e-5 and np.abs(got - want).max() <= 1e-4, f"{what}: rel rms {rel:.2e}"


@pytest.fixture(scope="module", params=["v2", "v2ProPlus"])
def setup(request):
    from genie_tts_amd.engine import Engine
    from oracle import restate as R
    ver = request.param
    w = character(ver)
    groups = {k: w[k] for k in ("t2s_encoder", "t2s", "vits") if k in w}
    if "prompt_encoder" in w:
        groups["prompt_encoder"] = w["prompt_encoder"]
    e = Engine(groups, ver)
    vm = R.VitsModel(w["vits"], ver)
    yield ver, e, vm, w
    e.close()


def _cond(ver):
    if ver == "v2":
        return dict(ref_audio=synth.synth_ref_audio(32000 * 2 + 1234))
    return dict(ge=synth.synth_ge(1024), ge_advanced=synth.synth_ge(512, "adv"))


@pytest.mark.parametrize("G,S,noise", [(8, 10, False), (8, 10, True), (80, 45, True)])
def test_vits_waveform(setup, G, S, noise):
    ver, e, vm, _ = setup
    txt = synth.synth_phones(S, f"vt{S}")
    sem = ((np.arange(G, dtype=np.int64) * 37 + 11) % 1024).reshape(1, 1, G)
    eps = synth.rng_for(f"eps{G}").standard_normal((1, 192, 2 * G)).astype(np.float32) if noise else None
    kw = _cond(ver)
    ref = vm(txt, sem, eps=eps, **kw).numpy()
    out = e.vits_decode(txt, sem, eps=eps, **kw).cpu().numpy()
    assert out.shape == (1280 * G,) == ref.shape
    rms = float(np.sqrt(np.mean((out - ref) ** 2)))
    assert rms <= RMS_TOL, f"rms {rms:.3e} (signal rms {np.sqrt(np.mean(ref**2)):.3e})"
    assert np.abs(out - ref).max() < 2e-3


@pytest.mark.parametrize("convh,fused", [(0, 0), (1, 0), (1, 1)])
def test_vits_waveform_conv_paths(setup, convh, fused):
    """MRF convs on the f32 MFMA path (convh=0) and on the f16-split path (1, default);
    on the latter the C <= 32 stages' conv pairs run separately (mrf_fused=0) or as one
    kernel with the intermediate in LDS (1, default, vits_mrf.hip)."""
    ver, e, vm, _ = setup
    G, S = 40, 30
    txt = synth.synth_phones(S, f"vt{S}")
    sem = ((np.arange(G, dtype=np.int64) * 53 + 7) % 1024).reshape(1, 1, G)
    eps = synth.rng_for(f"eps{G}").standard_normal((1, 192, 2 * G)).astype(np.float32)
    kw = _cond(ver)
    ref = vm(txt, sem, eps=eps, **kw).numpy()
    e.set_option("convh", convh)
    e.set_option("mrf_fused", fused)
    try:
        out = e.vits_decode(txt, sem, eps=eps, **kw).cpu().numpy()
    finally:
        e.set_option("convh", 1)
        e.set_option("mrf_fused", 1)
    rms = float(np.sqrt(np.mean((out - ref) ** 2)))
    assert rms <= RMS_TOL, f"rms {rms:.3e}"


def test_vits_fp16_range_guard_reruns_f32(setup):
    """An MRF conv input beyond the fp16 range (|x| > 65504, `vits_convh.hip` range guard)
    re-runs the utterance on the f32 path: the audio equals the convh=0 path's and the
    `vits_f32_reruns` counter moves.  Huge noise (eps x 1e6) drives the activations there."""
    ver, e, _, _ = setup
    G, S = 24, 16
    txt = synth.synth_phones(S, f"vt{S}")
    sem = ((np.arange(G, dtype=np.int64) * 29 + 5) % 1024).reshape(1, 1, G)
    eps = (synth.rng_for(f"big{G}").standard_normal((1, 192, 2 * G)) * 1e6).astype(np.float32)
    kw = _cond(ver)
    n0 = e.counter("vits_f32_reruns")
    out = e.vits_decode(txt, sem, eps=eps, **kw).cpu().numpy()
    assert e.counter("vits_f32_reruns") == n0 + 1
    e.set_option("convh", 0)
    try:
        ref = e.vits_decode(txt, sem, eps=eps, **kw).cpu().numpy()
    finally:
        e.set_option("convh", 1)
    assert np.isfinite(out).all()
    assert np.array_equal(out, ref)
    # normal inputs stay on the fp16-split path
    e.vits_decode(txt, sem, eps=eps * 1e-6, **kw)
    assert e.counter("vits_f32_reruns") == n0 + 1


@pytest.mark.parametrize("seg", [0, 1])
def test_vits_batch_range_guard_reruns_only_that_item(setup, seg):
    """Batched vocoder (`gsv_vits_decode_batch`) with an item whose MRF inputs leave the fp16
    range.  Per-lane passes (seg_vocoder 0): only that item re-runs on the f32 path and
    every item equals its single call bit for bit.  Segmented batch (1, default): the
    batch's one generator pass re-runs on the f32 path; every item matches its single
    call (the big one: the f32 path's)."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    items = []
    for i, (G, S, big) in enumerate([(16, 12, False), (24, 16, True), (20, 14, False)]):
        eps = synth.rng_for(f"bb{i}").standard_normal((1, 192, 2 * G)).astype(np.float32)
        items.append(dict(text_seq=synth.synth_phones(S, f"bb{S}"),
                          pred_semantic=((np.arange(G, dtype=np.int64) * 31 + i) % 1024).reshape(1, 1, G),
                          eps=eps * (1e6 if big else 1.0), **kw))
    n0 = e.counter("vits_f32_reruns")
    e.set_option("seg_vocoder", seg)
    try:
        outs = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    finally:
        e.set_option("seg_vocoder", 1)
    assert e.counter("vits_f32_reruns") == n0 + 1
    for i, (it, o) in enumerate(zip(items, outs)):
        single = e.vits_decode(it["text_seq"], it["pred_semantic"], eps=it["eps"], **kw).cpu().numpy()
        if seg == 0:
            assert np.array_equal(o, single)
        else:
            assert np.isfinite(o).all()
            _close(o, single, f"item {i}")


def test_vits_async_range_guard_reruns_f32(setup):
    """Overlapped vocoder call (`gsv_vits_decode_async` on the vocoder CUs): past the fp16 range
    it re-runs on the f32 path inside `gsv_vits_wait`; audio equals the single call's."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    G, S = 24, 16
    it = dict(text_seq=synth.synth_phones(S, f"va{S}"),
              pred_semantic=((np.arange(G, dtype=np.int64) * 13 + 3) % 1024).reshape(1, 1, G),
              eps=(synth.rng_for("vabig").standard_normal((1, 192, 2 * G)) * 1e6).astype(np.float32), **kw)
    single = e.vits_decode(it["text_seq"], it["pred_semantic"], eps=it["eps"], **kw).cpu().numpy()
    n0 = e.counter("vits_f32_reruns")
    e.set_vocoder_cus(64)
    try:
        audio = e.vits_decode_async(it)
        e.vits_wait()
        got = audio.cpu().numpy()
    finally:
        e.set_vocoder_cus(0)
    assert e.counter("vits_f32_reruns") == n0 + 1
    assert np.array_equal(got, single)


def test_prompt_encoder(setup):
    ver, e, _, w = setup
    if ver == "v2":
        pytest.skip("prompt encoder is V2ProPlus only")
    from oracle import restate as R
    ra = synth.synth_ref_audio(32000 * 3)
    sv = synth.rng_for("sv").standard_normal((1, 20480)).astype(np.float32)
    ge, ga = e.prompt_encode(ra, sv)
    ge_r, ga_r = R.prompt_encoder(w["prompt_encoder"], ra, sv)
    np.testing.assert_allclose(ge.cpu().numpy(), ge_r.numpy().reshape(-1), atol=2e-4, rtol=1e-4)
    np.testing.assert_allclose(ga.cpu().numpy(), ga_r.numpy().reshape(-1), atol=2e-4, rtol=1e-4)


def test_vits_philox_noise(setup):
    """Device Philox eps (noise_seed, the reference's RandomNormalLike x 0.5 default) vs
    the oracle fed the same stream restated in numpy (tests/philox.py)."""
    from tests.philox import vits_noise
    ver, e, vm, _ = setup
    G, S, seed = 30, 20, 0xC0FFEE
    txt = synth.synth_phones(S, f"vt{S}")
    sem = ((np.arange(G, dtype=np.int64) * 29 + 5) % 1024).reshape(1, 1, G)
    kw = _cond(ver)
    eps = vits_noise(192 * 2 * G, seed).reshape(1, 192, 2 * G)
    ref = vm(txt, sem, eps=eps, **kw).numpy()
    out = e.vits_decode(txt, sem, noise_seed=seed, **kw).cpu().numpy()
    rms = float(np.sqrt(np.mean((out - ref) ** 2)))
    assert rms <= RMS_TOL, f"rms {rms:.3e}"
    zero = e.vits_decode(txt, sem, **kw).cpu().numpy()
    assert np.sqrt(np.mean((zero - out) ** 2)) > 10 * RMS_TOL      # the noise is really applied


@pytest.mark.parametrize("seg", [0, 1])
def test_vits_batch_lanes_match_single(setup, seg):
    """gsv_vits_decode_batch for mixed lengths and noise modes.  seg_vocoder 0: the
    utterances on concurrent lanes with their own workspaces give the single-call
    results bit for bit.  seg_vocoder 1 (default): front parts on the lanes, then one
    generator pass over the batch laid out back to back with zero gaps (ConvArgs::seg):
    each utterance matches its single call to fp32 rounding, and the oracle within the
    north-star bar."""
    ver, e, vm, _ = setup
    kw = _cond(ver)
    items, singles = [], []
    for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9), (47, 31), (26, 18), (40, 40)]):
        txt = synth.synth_phones(S, f"vb{i}")
        sem = ((np.arange(G, dtype=np.int64) * (7 + i) + 3 * i) % 1024).reshape(1, 1, G)
        it = dict(text_seq=txt, pred_semantic=sem, **kw)
        if i % 3 == 1:
            it["noise_seed"] = 1000 + i
        elif i % 3 == 2:
            it["eps"] = synth.rng_for(f"vbe{i}").standard_normal((1, 192, 2 * G)).astype(np.float32)
        items.append(it)
        singles.append(e.vits_decode(txt, sem, eps=it.get("eps"), noise_seed=it.get("noise_seed"),
                                     **kw).cpu().numpy())
    e.set_option("seg_vocoder", seg)
    try:
        outs = e.vits_decode_batch(items)
    finally:
        e.set_option("seg_vocoder", 1)
    for i, (o, s1) in enumerate(zip(outs, singles)):
        if seg == 0:
            np.testing.assert_array_equal(o.cpu().numpy(), s1, err_msg=f"item {i}")
        else:
            _close(o.cpu().numpy(), s1, f"item {i}")
    if seg:
        it = items[2]
        ref = vm(it["text_seq"], it["pred_semantic"], eps=it["eps"], **kw).numpy().reshape(-1)
        assert float(np.sqrt(np.mean((outs[2].cpu().numpy() - ref) ** 2))) <= RMS_TOL


def test_convt_split_tile_ks4_on_concurrent_lanes(setup):
    """r04's nondeterminism, pinned: the upsample ConvTransposes on the split-fp16 path with
    every k_conv_h forced to the four-way K-split tile (1,1,4) -- the tile whose polyphase
    instance hipcc built with an op_sel'd v_pk_mul_f32 that gfx950 corrupted beside MFMA
    work (build.py, tests/test_isa_audit.py).  Six utterances on four concurrent lanes,
    ten batches: every utterance equals its single call bit for bit (r04u: 5 of 60 wrong)."""
    ver, e, vm, _ = setup
    kw = _cond(ver)
    items = []
    for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9), (47, 31), (26, 18), (40, 40)]):
        txt = synth.synth_phones(S, f"vk{i}")
        sem = ((np.arange(G, dtype=np.int64) * (5 + i) + 7 * i) % 1024).reshape(1, 1, G)
        it = dict(text_seq=txt, pred_semantic=sem, **kw)
        if i % 2:
            it["noise_seed"] = 2000 + i
        items.append(it)
    e.set_option("convt_f16", 1)
    e.set_option("convh_tile", 3)
    try:
        singles = [e.vits_decode(it["text_seq"], it["pred_semantic"], noise_seed=it.get("noise_seed"),
                                 **kw).cpu().numpy() for it in items]
        e.set_option("seg_vocoder", 0)
        wrong = []
        for rep in range(10):
            outs = e.vits_decode_batch(items)
            wrong += [(rep, i) for i, (o, s1) in enumerate(zip(outs, singles))
                      if not np.array_equal(o.cpu().numpy(), s1)]
    finally:
        e.set_option("seg_vocoder", 1)
        e.set_option("convh_tile", 0)
    assert not wrong, f"lanes differ from single calls: {wrong}"
    # and the forced tile is the same function as the cost model's tiles (oracle bar)
    ref = vm(items[2]["text_seq"], items[2]["pred_semantic"], **kw).numpy().reshape(-1)
    assert float(np.sqrt(np.mean((singles[2] - ref) ** 2))) <= RMS_TOL


def test_vits_batch_async_beside_t2s(setup):
    """gsv_vits_decode_batch_async: the lanes run while a batched T2S generate is issued
    on the engine stream (the pipelined batch mode); audio equals the joined batch call
    bit for bit and the T2S tokens equal those of the same generate run alone."""
    from genie_tts_amd import workloads
    from genie_tts_amd.engine import make_sampler
    ver, e, _, _ = setup
    kw = _cond(ver)
    items = []
    for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9), (47, 31), (26, 18), (40, 40), (12, 7)]):
        txt = synth.synth_phones(S, f"va{i}")
        sem = ((np.arange(G, dtype=np.int64) * (5 + i) + 2 * i) % 1024).reshape(1, 1, G)
        items.append(dict(text_seq=txt, pred_semantic=sem, noise_seed=2000 + i, **kw))
    ref_audio = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    wl = workloads.batch64(12, tag="vba")
    r = wl.reference
    utts = [(r.ref_seq, it.text_seq, None, None, r.ssl.reshape(768, -1), it.force_steps) for it in wl.items]
    sp = make_sampler(top_k=5, greedy=False, seed=0xBA7C)
    ref_tok = [t.tolist() for t in e.t2s_generate(utts, sp)]
    for _ in range(2):
        outs = e.vits_decode_batch_async(items)
        tok = [t.tolist() for t in e.t2s_generate(utts, sp)]
        e.vits_batch_wait()
        assert tok == ref_tok
        for i, (o, a) in enumerate(zip(outs, ref_audio)):
            np.testing.assert_array_equal(o.cpu().numpy(), a, err_msg=f"item {i}")
    # a synchronous vocoder call while a batch is pending finishes the batch first
    outs = e.vits_decode_batch_async(items)
    one = e.vits_decode(items[0]["text_seq"], items[0]["pred_semantic"], noise_seed=2000, **kw).cpu().numpy()
    _close(one, ref_audio[0], "single vs segmented batch")
    e.vits_batch_wait()
    np.testing.assert_array_equal(outs[-1].cpu().numpy(), ref_audio[-1])


def test_v2_ref_encode_once(setup):
    """gsv_ref_encode: the V2 vocoder's reference branch computed once and passed as ge
    gives the same audio, bit for bit, as passing the reference audio to every call
    (per-lane front parts); with ge the batch's front part runs packed (seg_front), which
    matches to fp32 rounding, and the overlapped batch gives the joined batch's audio bit
    for bit; V2ProPlus rejects it."""
    from genie_tts_amd.engine import EngineError
    ver, e, _, _ = setup
    kw = _cond(ver)
    if ver != "v2":
        with pytest.raises(EngineError, match="prompt_encode"):
            e.ref_encode(synth.synth_ref_audio(32000 * 2 + 1234))
        return
    ge = e.ref_encode(kw["ref_audio"])
    assert ge.shape == (512,)
    items = []
    for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9)]):
        txt = synth.synth_phones(S, f"vr{i}")
        sem = ((np.arange(G, dtype=np.int64) * (3 + i) + i) % 1024).reshape(1, 1, G)
        items.append(dict(text_seq=txt, pred_semantic=sem, noise_seed=77 + i))
    ref = [o.cpu().numpy() for o in e.vits_decode_batch([dict(it, **kw) for it in items])]
    e.set_option("seg_front", 0)
    try:
        lanes = [o.cpu().numpy() for o in e.vits_decode_batch([dict(it, ge=ge) for it in items])]
    finally:
        e.set_option("seg_front", 1)
    got = [o.cpu().numpy() for o in e.vits_decode_batch([dict(it, ge=ge) for it in items])]
    one = e.vits_decode(items[1]["text_seq"], items[1]["pred_semantic"], noise_seed=78, ge=ge).cpu().numpy()
    outs = e.vits_decode_batch_async([dict(it, ge=ge) for it in items])
    e.vits_batch_wait()
    for i in range(3):
        np.testing.assert_array_equal(lanes[i], ref[i])
        _close(got[i], ref[i], f"packed front, item {i}")
        np.testing.assert_array_equal(outs[i].cpu().numpy(), got[i])
    _close(one, ref[1], "single vs segmented batch")


def test_vits_segmented_batch_many_utterances(setup):
    """A segmented batch larger than the lane count, with a 1-token utterance, equal
    lengths and the longest one last: every utterance matches its single call, and the
    gaps between utterances stay zero (no audio leaks from a neighbour)."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    items = []
    for i, G in enumerate([1, 17, 17, 5, 60, 3, 29, 90]):
        S = 6 + (i * 5) % 30
        items.append(dict(text_seq=synth.synth_phones(S, f"vs{i}"),
                          pred_semantic=((np.arange(G, dtype=np.int64) * (11 + i) + i) % 1024).reshape(1, 1, G),
                          noise_seed=500 + i, **kw))
    outs = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    for i, it in enumerate(items):
        single = e.vits_decode(it["text_seq"], it["pred_semantic"], noise_seed=it["noise_seed"], **kw).cpu().numpy()
        _close(outs[i], single, f"item {i}")


def test_vits_batch_packed_front_matches_single(setup):
    """Segmented batch with the text/flow part packed too (option seg_front, the default when
    every item carries its conditioning vectors and noise_mode 0 or 2): the utterances back
    to back along the frame and text axes with zero gaps, self-attention (rel-pos) and the
    MRTE cross-attention within each utterance, per-utterance ge / Philox keys.  Each item
    matches its single call to fp32 rounding, the per-lane fronts (seg_front 0) too, the
    zero-noise item the oracle within the north-star bar, and the packed path really ran
    (counter vits_packed_fronts)."""
    ver, e, vm, _ = setup
    kw0 = _cond(ver)
    kw = dict(ge=e.ref_encode(kw0["ref_audio"])) if ver == "v2" else kw0   # (gsv_ref_encode, as the API does)
    items = []
    for i, (G, S) in enumerate([(20, 12), (33, 25), (8, 9), (47, 31), (26, 18), (40, 40), (3, 2)]):
        txt = synth.synth_phones(S, f"vp{i}")
        sem = ((np.arange(G, dtype=np.int64) * (11 + i) + 5 * i) % 1024).reshape(1, 1, G)
        it = dict(text_seq=txt, pred_semantic=sem, **kw)
        if i % 2 == 0:
            it["noise_seed"] = 3000 + i
        items.append(it)
    singles = [e.vits_decode(it["text_seq"], it["pred_semantic"], noise_seed=it.get("noise_seed"), **kw).cpu().numpy()
               for it in items]
    n0 = e.counter("vits_packed_fronts")
    packed = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    assert e.counter("vits_packed_fronts") == n0 + 1
    e.set_option("seg_front", 0)
    try:
        lanes = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    finally:
        e.set_option("seg_front", 1)
    assert e.counter("vits_packed_fronts") == n0 + 1
    for i, (p, l, s1) in enumerate(zip(packed, lanes, singles)):
        _close(p, s1, f"item {i} vs single")
        _close(p, l, f"item {i} vs lane fronts")
    it = items[1]   # no noise: the oracle directly
    ref = vm(it["text_seq"], it["pred_semantic"], **kw0).numpy().reshape(-1)
    assert float(np.sqrt(np.mean((packed[1] - ref) ** 2))) <= RMS_TOL


@pytest.mark.parametrize("seg", [1, 0])
def test_vits_batch_persistent_convs_bit_identical(setup, seg):
    """Option convh_persist: the batch's large split-fp16 MRF convs and ConvTransposes run as a
    persistent tile loop (two blocks per CU walking the output tiles, the next tile's first chunk
    staged during the current tile's last; vits_convh.hip PERS).  Every tile runs the one-block
    kernel's MFMA sequence, so the batch's audio is bit-identical with the option on and off --
    on the segmented generator (seg 1: its stages 2-3 have > 2048 tiles) and on per-utterance
    lanes (seg 0)."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    items = []
    for i in range(14):
        G, S = 70 + 5 * i, 30 + i
        txt = synth.synth_phones(S, f"vp{i}")
        sem = ((np.arange(G, dtype=np.int64) * (11 + i) + 5 * i) % 1024).reshape(1, 1, G)
        items.append(dict(text_seq=txt, pred_semantic=sem, noise_seed=3000 + i, **kw))
    e.set_option("seg_vocoder", seg)
    try:
        want = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
        e.set_option("convh_persist", 1)
        got = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    finally:
        e.set_option("convh_persist", 0)
        e.set_option("seg_vocoder", 1)
    for i, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g, w, err_msg=f"item {i}")


def test_vits_batch_weight_stationary_convs_bit_identical(setup):
    """Option convh_ws: the segmented generator's 7- / 11-tap MRF convs with 64 input channels and
    its 7-tap ones with 128 run as k_conv_ws -- a block keeps its 64 output channels'
    weights in LDS and walks 256-column tiles (vits_convh.hip).  Each accumulator runs k_conv_h's
    MFMA sequence, so the batch's audio is bit-identical with the option on and off."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    items = []
    for i in range(14):
        G, S = 70 + 5 * i, 30 + i
        txt = synth.synth_phones(S, f"vw{i}")
        sem = ((np.arange(G, dtype=np.int64) * (13 + i) + 7 * i) % 1024).reshape(1, 1, G)
        items.append(dict(text_seq=txt, pred_semantic=sem, noise_seed=4000 + i, **kw))
    try:
        e.set_option("convh_ws", 0)
        want = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
        e.set_option("convh_ws", 1)
        got = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
        e.set_option("convh_ws", 2)   # the default: a synchronous batch runs the form too
        got2 = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
    finally:
        e.set_option("convh_ws", 2)
    for i, (g, w) in enumerate(zip(got2, want)):
        np.testing.assert_array_equal(g, w, err_msg=f"item {i} (default)")
    for i, (g, w) in enumerate(zip(got, want)):
        np.testing.assert_array_equal(g, w, err_msg=f"item {i}")


def test_vits_front_text_branch_on_the_side_stream_bit_identical(setup):
    """Option vits_fork (default 1): the front's text branch (embedding, encoder_text, MRTE text_pre /
    k-v) runs on a side stream beside the SSL branch and joins before MRTE's attention
    (vits_front).  Same kernels and buffers of its own: one utterance's audio and a packed batch's
    are bit-identical with the fork on and off."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    txt = synth.synth_phones(37, "vf")
    sem = ((np.arange(61, dtype=np.int64) * 29 + 3) % 1024).reshape(1, 1, 61)
    items = []
    for i in range(5):
        G, S = 30 + 9 * i, 14 + 5 * i
        t = synth.synth_phones(S, f"vfb{i}")
        sm = ((np.arange(G, dtype=np.int64) * (17 + i) + i) % 1024).reshape(1, 1, G)
        items.append(dict(text_seq=t, pred_semantic=sm, noise_seed=5000 + i, **kw))
    out = {}
    try:
        for f in (1, 0):
            e.set_option("vits_fork", f)
            one = e.vits_decode(txt, sem, noise_seed=77, **kw).cpu().numpy()
            batch = [o.cpu().numpy() for o in e.vits_decode_batch(items)]
            out[f] = (one, batch)
    finally:
        e.set_option("vits_fork", 1)
    np.testing.assert_array_equal(out[1][0], out[0][0])
    for i, (a, b) in enumerate(zip(out[1][1], out[0][1])):
        np.testing.assert_array_equal(a, b, err_msg=f"item {i}")


def test_vits_fork_survives_stream_remakes(setup):
    """The fork's side streams are made beside the engine stream and dropped whenever the engine
    re-makes its streams (option vocoder_cus): a forked single call, then the CU split on and an
    overlapped call (masked stream: no fork), then the split off and a forked call again -- every
    result equals the first, bit for bit."""
    ver, e, _, _ = setup
    kw = _cond(ver)
    txt = synth.synth_phones(29, "vr")
    sem = ((np.arange(53, dtype=np.int64) * 31 + 5) % 1024).reshape(1, 1, 53)
    first = e.vits_decode(txt, sem, noise_seed=91, **kw).cpu().numpy()
    try:
        e.set_vocoder_cus(64)
        out = e.vits_decode_async(dict(text_seq=txt, pred_semantic=sem, noise_seed=91, **kw))
        e.vits_wait()
        np.testing.assert_array_equal(out.cpu().numpy(), first)
    finally:
        e.set_vocoder_cus(0)
    again = e.vits_decode(txt, sem, noise_seed=91, **kw).cpu().numpy()
    np.testing.assert_array_equal(again, first)
