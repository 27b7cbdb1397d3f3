"""GPU: the engine's device footprint stays bounded under a server-style load ramp
(ADVICE r05 engine.hip:373).

A server worker decodes every ready sentence of a round in one generate (server.py
round_size), with the reference's unforced sampler (max_steps 500, Inference.py:95-106), so
the batch grows 1 -> 64 and the prompt length n0 creeps up as longer sentences arrive.  Each
new maximum used to re-allocate the KV cache, the persistent ring and the packed-prefill
buffers at exactly the new size and keep the old ones until the engine was destroyed
(retired, not freed: a hipFree beside another thread's capture invalidates it).
Now capacities grow in quantised steps and the growth path frees the retired buffers once
the engine's own streams drained (gsv_engine::reclaim, under the process-wide capture lock).

Bar: after the ramp, the engine's share of the device (hipMemGetInfo via
torch.cuda.mem_get_info) is at most 1.5x that of a fresh engine that ran only the ramp's
last round, nothing retired is left unfreed, and the tokens of the last round equal the
fresh engine's.  The reference re-creates ORT buffers per call (ModelManager.py:59-114,
Inference.py:98-103) and never accumulates.
"""
import numpy as np
import pytest

from genie_tts_amd import synth
from tests.common import character

pytestmark = pytest.mark.gpu

RAMP = [1, 2, 3, 5, 8, 12, 17, 24, 33, 47, 64]


def _round(torch, B, k):
    """B sentences; the prompt (reference + text + ssl) grows with the round index k."""
    T = lambda a: torch.as_tensor(a, device="cuda")
    out = []
    for i in range(B):
        ref = synth.synth_phones(12 + 6 * k, f"mr{k}")
        txt = synth.synth_phones(8 + 4 * k + (i % 5), f"mt{k}.{i}")
        ssl = synth.synth_ssl(40 + 24 * k, f"ms{k}").reshape(768, -1)
        out.append((T(ref), T(txt), None, None, T(ssl)))
    return out


def _used(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    return free


def test_footprint_bounded_under_a_batch_and_length_ramp():
    import torch
    from genie_tts_amd.engine import Engine, make_sampler
    ch = {k: v for k, v in character("v2").items() if k in ("t2s_encoder", "t2s")}
    sp = make_sampler(max_steps=500)   # the reference's loop bound, no forced length
    rounds = [_round(torch, B, k) for k, B in enumerate(RAMP)]

    free0 = _used(torch)
    e = Engine(ch, "v2")
    try:
        for utts in rounds:
            toks_ramp = e.t2s_generate(utts, sp)
        used_ramp = free0 - _used(torch)
        retired = e.counter("retired_bytes")
        reclaimed, reclaims = e.counter("reclaimed_bytes"), e.counter("reclaims")
    finally:
        e.close()

    free1 = _used(torch)
    f = Engine(ch, "v2")
    try:
        toks_fresh = f.t2s_generate(rounds[-1], sp)
        used_fresh = free1 - _used(torch)
    finally:
        f.close()

    print(f"ramp {used_ramp / 2**30:.2f} GiB, fresh {used_fresh / 2**30:.2f} GiB, "
          f"reclaimed {reclaimed / 2**30:.2f} GiB in {reclaims} passes, retired left {retired}")
    assert len(toks_ramp) == len(toks_fresh) == RAMP[-1]
    for a, b in zip(toks_ramp, toks_fresh):
        np.testing.assert_array_equal(a, b)
    assert retired == 0
    assert reclaims > 0 and reclaimed > 0
    assert used_ramp <= 1.5 * used_fresh, (used_ramp, used_fresh)
