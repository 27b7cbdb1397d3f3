"""CPU: replica sharding -- LPT plan and the world_size-2 gloo path.

The synthesis function here is a host stand-in (the engine needs a GPU); what
is under test is the plan and the in-order gather that the 8-GPU run relies on.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from genie_tts_amd.replicas import Request, lpt_assign, predicted_cost, run_sharded


def test_lpt_plan_is_a_balanced_partition():
    rng = np.random.default_rng(3)
    costs = rng.uniform(30, 170, size=100).tolist()
    for n in (1, 2, 4, 8):
        shards = lpt_assign(costs, n)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(100))
        loads = [sum(costs[i] for i in s) for s in shards]
        # Graham's LPT bound: makespan <= 4/3 OPT, and OPT >= mean load
        assert max(loads) <= (4 / 3) * max(sum(costs) / n, max(costs)) + 1e-9
    assert lpt_assign(costs, 8) == lpt_assign(list(costs), 8)     # deterministic on every rank


def test_predicted_cost_orders_by_length():
    a = Request(0, np.arange(20))
    b = Request(1, np.arange(60))
    assert predicted_cost(b) > predicted_cost(a)
    assert predicted_cost(Request(2, np.arange(20), force_steps=200)) > predicted_cost(b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    reqs = [Request(i, np.arange(10 + (i * 7) % 50)) for i in range(23)]
    seen = []

    def synth(rs):
        seen.extend(r.idx for r in rs)
        return [np.full(r.n_phones, r.idx, np.int32) for r in rs]
    out = run_sharded(reqs, synth, rank, world)
    q.put((rank, sorted(seen), None if out is None else [(int(o[0]), o.size) for o in out]))
    dist.destroy_process_group()


def test_gloo_world2_gather_in_order():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        rank, seen, out = q.get(timeout=120)
        res[rank] = (seen, out)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(res[0][0] + res[1][0]) == list(range(23))      # every request exactly once
    assert res[0][0] and res[1][0]                                 # both ranks got work
    assert res[1][1] is None
    assert [i for i, _ in res[0][1]] == list(range(23))
    assert [n for _, n in res[0][1]] == [10 + (i * 7) % 50 for i in range(23)]
