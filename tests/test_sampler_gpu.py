"""GPU: the decode sampler kernel (K10, stage#1775-1806) against the oracle's
`sample` (oracle/restate.py) on identical logits, histories and noise.

Bar: identical token ids and stop flags.  Covers greedy (q := 1) and sampled
(q = Philox/Box-Muller, tests/philox.py) modes, top-k 1/5/15/64,
temperature, repetition penalty, and ties at the top-k threshold (multiplicity).
"""
import numpy as np
import pytest
import torch

from tests.philox import sampler_noise

pytestmark = pytest.mark.gpu


def _seen_bits(hist):
    bits = np.zeros(33, np.uint32)
    for t in hist:
        bits[t >> 5] |= np.uint32(1 << (t & 31))
    return bits.view(np.int32)


@pytest.mark.parametrize("top_k,temp,greedy", [(15, 1.0, True), (15, 1.0, False), (5, 0.7, False),
                                               (1, 1.0, False), (64, 1.3, False), (15, 1.0, False)])
def test_sampler_matches_oracle(top_k, temp, greedy):
    from genie_tts_amd.engine import debug_sample, make_sampler
    from oracle import restate as R
    rng = np.random.default_rng(top_k * 100 + int(temp * 10) + greedy)
    B, step, seed = 7, 13, 0x1234_5678_9ABC
    logits = rng.normal(0, 3, size=(B, 1025)).astype(np.float32)
    logits[2, :40] = logits[2].max() + 1.0          # many equal maxima
    logits[3, 100:130] = 2.5                         # a tie block straddling the top-k threshold
    logits[3, 500:505] = 9.0
    logits[4, 1024] = logits[4].max() + 5.0          # EOS wins the raw argmax -> stop
    hists = [rng.choice(1025, size=int(rng.integers(0, 200)), replace=False) for _ in range(B)]
    seen = np.stack([_seen_bits(h) for h in hists])
    sp = make_sampler(top_k=top_k, temperature=temp, greedy=greedy, seed=seed)
    tok, stop = debug_sample(torch.from_numpy(logits).cuda(), torch.from_numpy(seen).cuda(), sp, step)
    tok, stop = tok.cpu().numpy(), stop.cpu().numpy()
    cfg = R.SamplerCfg(top_k=top_k, temperature=temp)
    for b in range(B):
        q = torch.ones(1025) if greedy else torch.from_numpy(sampler_noise(1025, step, b, seed))
        t_ref, raw = R.sample(torch.from_numpy(logits[b]), torch.as_tensor(np.asarray(hists[b], np.int64)), q, cfg)
        assert int(tok[b]) == t_ref, (b, int(tok[b]), t_ref)
        assert bool(stop[b]) == (raw == 1024 or t_ref == 1024)


def test_top_k_out_of_range_is_an_error():
    from genie_tts_amd.engine import EngineError, debug_sample, make_sampler
    lg = torch.zeros((1, 1025), device="cuda")
    seen = torch.zeros((1, 33), dtype=torch.int32, device="cuda")
    with pytest.raises(EngineError):
        debug_sample(lg, seen, make_sampler(top_k=65), 1)
