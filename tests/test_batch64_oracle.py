"""CPU: pin tests/golden/t2s_batch64.npz to the oracle (oracle/restate.py) on a
few utterances of each sampler mode, and check the workload definition the
fixture was generated from is unchanged."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "t2s_batch64.npz")


def test_workload_shape():
    from genie_tts_amd import workloads
    g = np.load(GOLD)
    wl = workloads.batch64()
    assert len(wl.items) == 64
    assert [it.text_seq.shape[1] for it in wl.items] == g["S"].tolist()
    assert [it.tokens for it in wl.items] == g["G"].tolist()
    assert all(30 <= s <= 60 for s in g["S"]) and all(50 <= x <= 110 for x in g["G"])


@pytest.mark.parametrize("b,greedy", [(0, True), (33, True), (5, False), (63, False)])
def test_fixture_rows_match_oracle(b, greedy):
    from tests.golden.make_batch64 import oracle_tokens
    g = np.load(GOLD)
    key = "greedy" if greedy else "topk"
    ref = g[key][b, :g[key + "_len"][b]].astype(np.int64)
    assert oracle_tokens(b, greedy).tolist() == ref.tolist()
