"""Multi-GPU synthesis as independent replicas.

Utterances are independent: one process per GPU, each with a full engine
(weights ~0.3 GB, trivial against 288 GB), no collective on the data path
(xGMI/RCCL unused).  The host predicts each request's cost, assigns requests
to ranks by LPT (longest processing time first onto the least-loaded rank),
every rank synthesises its shard (batched through the engine), and results go
back to rank 0 in request order over a host-side gloo group -- PCM bytes, not
device tensors.

Cost model: T2S decode dominates and the semantic length grows with the
phoneme count (25 tokens/s of audio, ~2 tokens per phoneme for JP), so
cost ~ c0 + S (+ G when the caller knows it, e.g. a forced length).
"""
from __future__ import annotations

import heapq
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence


@dataclass
class Request:
    idx: int                      # position in the caller's order
    text_seq: object              # i64 [S] (or [1,S]) phoneme ids
    text_bert: object = None      # f32 [S,1024] or None (zeros, or RoBERTa below)
    force_steps: int = 0          # >0: known decode length (benchmarks)
    bert_ids: object = None       # Chinese: RoBERTa input_ids [C+2] (CLS .. SEP) ...
    word2ph: object = None        # ... and phones per character [C]: text_bert from RoBERTa

    @property
    def n_phones(self) -> int:
        import numpy as np
        return int(np.asarray(self.text_seq).size)


def predicted_cost(req: Request, c0: float = 8.0) -> float:
    g = req.force_steps if req.force_steps > 0 else 2 * req.n_phones
    return c0 + req.n_phones + g


def lpt_assign(costs: Sequence[float], n_ranks: int) -> List[List[int]]:
    """Greedy LPT: items sorted by cost (desc, ties by index) onto the least-loaded
    rank (ties by rank id).  Deterministic, so every rank computes the same plan."""
    if n_ranks < 1:
        raise ValueError("n_ranks must be >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, r) for r in range(n_ranks)]
    shards: List[List[int]] = [[] for _ in range(n_ranks)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    for s in shards:
        s.sort()
    return shards


def run_sharded(requests: Sequence[Request], synth: Callable[[List[Request]], List[object]], rank: int,
                world: int, group=None, gather: bool = True) -> Optional[List[object]]:
    """Synthesize this rank's shard with `synth(list_of_requests) -> list_of_outputs`.

    With world > 1 and gather=True, rank 0 receives every output in request
    order (torch.distributed.gather_object over `group`, which should be a
    gloo group: outputs are host arrays).  Other ranks return None."""
    shards = lpt_assign([predicted_cost(r) for r in requests], world)
    mine = [requests[i] for i in shards[rank]]
    outs = synth(mine) if mine else []
    if len(outs) != len(mine):
        raise RuntimeError(f"synth returned {len(outs)} outputs for {len(mine)} requests")
    local = list(zip([r.idx for r in mine], outs))
    if world == 1:
        return [o for _, o in sorted(local, key=lambda t: t[0])]
    if not gather:
        return [o for _, o in local]
    import torch.distributed as dist
    recv = [None] * world if rank == 0 else None
    dist.gather_object(local, recv, dst=0, group=group)
    if rank != 0:
        return None
    merged = [p for part in recv for p in part]
    merged.sort(key=lambda t: t[0])
    if [i for i, _ in merged] != sorted(r.idx for r in requests):
        raise RuntimeError("lost or duplicated requests in gather")
    return [o for _, o in merged]


def text_berts(reqs: Sequence[Request], roberta=None) -> List[object]:
    """Each request's BERT features: its text_bert, or -- a Chinese sentence given as
    RoBERTa inputs (bert_ids, word2ph) -- RoBERTa's, all such sentences of the list in one
    packed pass (`roberta.roberta_batch`, gsv_roberta_batch; the reference runs one
    RoBERTa session call per Chinese sentence, GetPhonesAndBert.py:64-74); else None
    (zeros: Japanese / English)."""
    out = [r.text_bert for r in reqs]
    zh = [i for i, r in enumerate(reqs) if r.text_bert is None and r.bert_ids is not None]
    if zh:
        if roberta is None:
            raise ValueError("Chinese requests given as RoBERTa inputs need a RoBERTa engine")
        feats = roberta.roberta_batch([(reqs[i].bert_ids, reqs[i].word2ph) for i in zh])
        for i, f in zip(zh, feats):
            out[i] = f
    return out


def engine_synth(model, reference, sampler_factory, roberta=None) -> Callable[[List[Request]], List[object]]:
    """synth() over one engine-backed GSVModel: the shard's Chinese BERT features
    (text_berts, on `roberta` -- an Engine holding RoBERTa weights, e.g. model.ENGINE),
    one batched T2S for the shard (each request's own forced length, if any), then the
    vocoder per utterance (inference.GENIE.tts_batch).  sampler_factory() -> engine.Sampler."""
    from .inference import tts_client

    def synth(reqs: List[Request]):
        items = [(r.text_seq, b, r.force_steps) for r, b in zip(reqs, text_berts(reqs, roberta))]
        return tts_client.tts_batch(items, reference, model, sampler_factory())
    return synth
