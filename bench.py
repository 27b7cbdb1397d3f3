#!/usr/bin/env python3
"""Benchmark: GPT-SoVITS inference (Genie hot path) on MI355X.

Metric (BASELINE.json): real-time factor + utterances/sec, 20-char JP, V2 speaker.

Workloads (genie_tts_amd/workloads.py; synthetic seeded inputs and synthetic
fp16-valued weights -- no checkpoints offline; random weights never emit EOS,
so every utterance runs a forced number of loop steps):
  single   (default, the headline line) configs[1]: one V2 utterance through the
           whole path -- T2S encoder, prefill, greedy decode (81 loop steps ->
           80 semantic tokens), VITS (ref STFT + MelStyleEncoder, TextEncoder,
           flow, HiFi-GAN) -> 102,400 samples = 3.2 s of 32 kHz audio.  R=48,
           S=45, H=264 (P=132 prompts), 5.3 s reference.  A step = one utterance
           of a stream of them (a paragraph split into sentences): each one's
           vocoder runs on --vocoder-cus CUs of its own (default 64) beside the
           next one's T2S on the other CUs (gsv_vits_decode_async); the line's
           "sequential" object times one utterance alone on every CU
           (--vocoder-cus 0 makes that the headline mode).
  batch64  configs[2]: 64 mixed-length JP sentences (S~U[30,60], G~U[50,110]),
           top-k 5 sampled, ONE ragged batched decode + the vocoder per
           utterance.  A step = the 64-sentence batch.
  mixed100 configs[3]: V2ProPlus EN+ZH 100-sentence set, LPT-sharded over the
           ranks (genie_tts_amd/replicas.py), each rank batching its shard; the
           Chinese sentences' BERT features come from RoBERTa (24-layer
           chinese-roberta-wwm-ext-large shapes, synthetic weights) on the engine,
           inside the timed region.  A step = the whole set (weak scaling does not
           apply: total work fixed).

Inputs are resident in HBM before the timed region.  Multi-GPU: one process per
GPU (torchrun), independent replicas, no collective on the data path; the
barrier and the max-over-ranks time use a gloo (host) group -- no RCCL.

The single workload's line also carries "concurrent_streams": the same stream run by two
child ranks sharing the GPU (each decoding on 96 CUs of its own, the vocoder CUs shared;
--streams-per-gpu), the GPU's rate under concurrent single-sentence requests.  The batched
workloads pipeline each batch's vocoder beside the next batch's T2S (--pipeline 0: one batch
at a time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload single|batch64|mixed100]
                       [--vocoder-cus K] [--concurrent-streams S] [--pipeline 0|1]
                       [--vits-lanes L] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "real-time factor + utterances/sec, 20-char JP, V2 speaker, 1/2/4/8 MI355X"
SR = 32000


def cpu_baseline(wl, threads: int):
    """Oracle restatement of Genie's ONNX-CPU path on the host cores (torch fp32),
    one utterance of the workload (bounded sample)."""
    import torch
    from genie_tts_amd import synth
    from oracle import restate as R
    torch.set_num_threads(threads)
    w = synth.synthetic_character("v2")
    m = R.T2SModel(w["t2s"])
    vm = R.VitsModel(w["vits"], "v2")
    ref, it = wl.reference, wl.items[0]
    tb = np.zeros((it.text_seq.shape[1], 1024), np.float32)
    t0 = time.perf_counter()
    sem, _, _ = R.t2s_generate(w["t2s_encoder"], m, ref.ref_seq, ref.ref_bert, it.text_seq, tb, ref.ssl,
                               force_steps=it.force_steps)
    wav = vm(it.text_seq, sem, ref_audio=ref.audio_32k)
    dt = time.perf_counter() - t0
    return dt, int(wav.numel())


class Runner:
    """One replica: engine + device-resident inputs of its share of the workload."""

    def __init__(self, wl, items, dev, device_index):
        import torch
        from genie_tts_amd import synth
        from genie_tts_amd.engine import Engine, make_sampler
        self.torch = torch
        self.wl = wl
        self.items = items
        w = synth.synthetic_character(wl.version)
        self.zh = any(it.bert_ids is not None for it in items)
        if self.zh:   # Chinese sentences: RoBERTa on the same engine (GetPhonesAndBert.py:64-74)
            from genie_tts_amd import workloads
            w["roberta"] = workloads.roberta_weights()
        self.eng = Engine(w, wl.version, device=device_index)
        ref = wl.reference
        T = lambda a, dt=None: torch.as_tensor(np.ascontiguousarray(a), device=dev)
        self.d_ref = T(ref.ref_seq.reshape(-1))
        self.d_ssl = T(ref.ssl.reshape(768, -1))
        self.d_audio = T(ref.audio_32k.reshape(-1))
        self.d_ref_bert = None if not np.any(ref.ref_bert) else T(ref.ref_bert)
        self.d_txt = [T(it.text_seq.reshape(-1)) for it in items]
        self.d_bert = [None if it.text_bert is None else T(it.text_bert) for it in items]
        self.d_bert_ids = [None if it.bert_ids is None else T(it.bert_ids) for it in items]
        self.sp = make_sampler(top_k=wl.top_k, greedy=wl.greedy)
        self.seed = 0x5EED
        self.ge = self.ge_adv = None
        if wl.version != "v2":
            self.ge, self.ge_adv = self.eng.prompt_encode(self.d_audio, T(ref.sv_emb.reshape(-1)))
        else:   # the vocoder's reference branch once per reference (gsv_ref_encode), as the API does
            self.ge_v2 = self.eng.ref_encode(self.d_audio)
        self.eng.set_option("persist", 1)
        self.phase = {"t2s": 0.0, "vits": 0.0, "encode+prefill": 0.0, "decode": 0.0, "roberta": 0.0}

    def stream(self, n, phase_ms=None):
        """n utterances as a pipelined stream: utterance i+1's T2S is queued behind
        utterance i's (gsv_t2s_generate_start / _finish, so the decode CUs never wait
        for the host), its encoder + prefill run on the vocoder CUs beside utterance
        i's decode (gsv_t2s_prefetch), and utterance i's vocoder runs there beside
        utterance i+1's decode (gsv_vits_decode_async)."""
        eng = self.eng
        if getattr(self, "utts", None) is None:
            # the stream's sentences are all the workload's one utterance, but each sentence
            # of a real stream has buffers of its own: alternate two copies, so sentence 0 is
            # not taken for the prefetched sentence 1 (its prefill runs on the T2S CUs, as
            # GENIE.tts_stream's first sentence does)
            self.utts = [(self.d_ref, t, self.d_ref_bert, self.d_bert[0], self.d_ssl, self.items[0].force_steps)
                         for t in (self.d_txt[0], self.d_txt[0].clone())]
        utt = lambda i: self.utts[i % 2]
        cond = dict(ge=self.ge_v2) if self.ge is None else dict(ge=self.ge, ge_advanced=self.ge_adv)
        if n > 1:
            eng.t2s_prefetch(utt(1), self.sp)   # launched beside sentence 0's decode
        eng.t2s_generate_start(utt(0), self.sp)
        sems = None
        for i in range(n):
            if i + 1 < n:
                if i + 2 < n:
                    eng.t2s_prefetch(utt(i + 2), self.sp)
                eng.t2s_generate_start(utt(i + 1), self.sp)
            sems = [eng.t2s_generate_finish()]
            if phase_ms is not None:
                phase_ms.append(eng.timing())
            self.finish()                                   # the previous utterance's vocoder
            self.pending = eng.vits_decode_async(dict(text_seq=utt(i)[1], pred_semantic=sems[0],
                                                      noise_seed=self.seed, **cond))
        self.finish()
        return sems, 1280 * int(sems[0].size)

    def finish(self):
        if getattr(self, "pending", None) is not None:
            self.eng.vits_wait()
            self.pending = None

    def berts(self, lo, hi):
        """BERT features of items [lo, hi): the Chinese ones from RoBERTa over their device
        token ids in one packed pass (gsv_roberta_batch) -- inside the timed region, as the
        reference runs RoBERTa per Chinese sentence on every tts call -- the rest as given."""
        out = self.d_bert[lo:hi]
        zh = [i for i in range(lo, hi) if self.d_bert_ids[i] is not None]
        if zh:
            t0 = time.perf_counter()
            feats = self.eng.roberta_batch([(self.d_bert_ids[i], self.items[i].word2ph) for i in zh])
            for i, f in zip(zh, feats):
                out[i - lo] = f
            self.phase["roberta"] = self.phase.get("roberta", 0.0) + time.perf_counter() - t0
        return out

    def step(self):
        torch = self.torch
        t0 = time.perf_counter()
        utts = [(self.d_ref, t, self.d_ref_bert, b, self.d_ssl, it.force_steps)
                for t, b, it in zip(self.d_txt, self.berts(0, len(self.items)), self.items)]
        sems = self.eng.t2s_generate(utts, self.sp)        # returns host tokens: synchronous
        t1 = time.perf_counter()
        tm = self.eng.timing()                              # device phases of this generate (ms)
        self.phase["encode+prefill"] += (tm[0] + tm[1]) * 1e-3
        self.phase["decode"] += tm[2] * 1e-3
        # vocoder with the reference's z_p noise (RandomNormalLike x 0.5) from the device Philox stream
        cond = dict(ge=self.ge_v2) if self.ge is None else dict(ge=self.ge, ge_advanced=self.ge_adv)
        if len(sems) == 1:
            wavs = [self.eng.vits_decode(self.d_txt[0], sems[0], noise_seed=self.seed, **cond)]
        else:   # concurrent vocoder lanes
            wavs = self.eng.vits_decode_batch([dict(text_seq=t, pred_semantic=sem, noise_seed=self.seed + i, **cond)
                                               for i, (t, sem) in enumerate(zip(self.d_txt, sems))])
        n = sum(int(w.numel()) for w in wavs)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        self.phase["t2s"] += t1 - t0
        self.phase["vits"] += t2 - t1
        return sems, n

    def step_pipelined(self):
        """One pass over the workload with the vocoder overlapped: the items go in balanced
        batches of <= 64 (the engine's decode batch); each batch's T2S runs beside the
        previous batch's vocoder lanes (gsv_vits_decode_batch_async), then that vocoder is
        joined and this batch's is started.  drain() joins the last one."""
        n = len(self.items)
        nb = -(-n // 64)
        bounds = [n * j // nb for j in range(nb + 1)]
        cond = dict(ge=self.ge_v2) if self.ge is None else dict(ge=self.ge, ge_advanced=self.ge_adv)
        sems_all, n_samples = [], 0
        for j in range(nb):
            lo, hi = bounds[j], bounds[j + 1]
            t0 = time.perf_counter()
            bert = self.berts(lo, hi)
            utts = [(self.d_ref, self.d_txt[i], self.d_ref_bert, bert[i - lo], self.d_ssl, self.items[i].force_steps)
                    for i in range(lo, hi)]
            sems = self.eng.t2s_generate(utts, self.sp)
            t1 = time.perf_counter()
            tm = self.eng.timing()
            self.phase["encode+prefill"] += (tm[0] + tm[1]) * 1e-3
            self.phase["decode"] += tm[2] * 1e-3
            self.drain()
            t2 = time.perf_counter()
            wavs = self.eng.vits_decode_batch_async(
                [dict(text_seq=self.d_txt[lo + i], pred_semantic=sem, noise_seed=self.seed + lo + i, **cond)
                 for i, sem in enumerate(sems)])
            self.batch_pending = True
            self.phase["t2s"] += t1 - t0
            self.phase["vits"] += t2 - t1      # the host's wait for the previous vocoder (not hidden)
            sems_all += sems
            n_samples += sum(int(w.numel()) for w in wavs)
        return sems_all, n_samples

    def drain(self):
        if getattr(self, "batch_pending", False):
            self.eng.vits_batch_wait()
            self.batch_pending = False


def concurrent_streams(args):
    """The single-utterance workload as S concurrent sentence streams on this one GPU: S
    child ranks (torch.distributed.run, gloo barrier + max time), each an engine whose
    persistent decode runs on 96 CUs of its own and whose vocoder + next prefill share the
    vocoder CUs.  Throughput of the GPU under concurrent single-utterance requests; the
    headline stays the single stream (north_star: single-stream real time)."""
    import socket
    import subprocess
    S = args.concurrent_streams
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={S}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__),
           "--streams-per-gpu", str(S), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--vocoder-cus", "64", "--decode-cus", "96", "--no-cpu-baseline"]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception as e:   # reported, never fatal to the headline line
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    return {"streams": S, "utt_s": d["value"], "x_realtime": d["value"] * d["audio_s_per_step"],
            "ms_per_utt_per_stream": d["ms_per_step"], "decode_cus_per_stream": 96, "vocoder_cus_shared": 64,
            "persist_timeouts": d["config"]["persist_timeouts"],
            "note": f"{S} sentence streams on one GPU, one rank each, decode CUs disjoint (CU-masked "
                    "persistent decode), vocoder + prefetch CUs shared"}


def launch_ranks(n: int, argv) -> int:
    """`--gpus N` run without a launcher (WORLD_SIZE unset): one rank per GPU as child
    processes of `torch.distributed.run`, started before this process touches the GPU
    (nothing is exec'd in place).  Their output is relayed line by line (rank 0 prints the
    JSON line); the exit code is theirs."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return p.wait()


class StubRunner:
    """CPU stand-in for Runner (tests of the multi-rank launcher and the max-over-ranks
    timing): a step sleeps `stub_ms`; no GPU, no engine."""

    def __init__(self, wl, items, stub_ms):
        self.items, self.ms = items, stub_ms
        self.phase = {}

    def step(self):
        time.sleep(self.ms * 1e-3)
        return [np.zeros(it.tokens, np.int64) for it in self.items], 1280 * sum(it.tokens for it in self.items)

    def drain(self):
        pass


def over_ranks(dist, dt: float, units: int):
    """(max wall time over the ranks, per-rank units/s) over the gloo group; (dt, [units/dt])
    without one.  The job's rate is every rank's units over the slowest rank's time."""
    if dist is None:
        return dt, [units / dt]
    import torch
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per = [None] * dist.get_world_size()
    dist.all_gather_object(per, units / dt)
    return float(t.item()), [float(x) for x in per]


def stub_main(args):
    """The multi-rank harness with StubRunner replicas (no GPU): gloo barrier, K timed
    steps, max over ranks, rank 0's JSON line -- what a GPU run reports, minus the engine."""
    from genie_tts_amd import workloads
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    wl = workloads.single()
    run = StubRunner(wl, wl.items, args.stub_ms * (1 + 0.5 * rank))   # uneven ranks: the max must win
    for _ in range(args.warmup):
        run.step()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, n_samples = run.step()
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    dt, per = over_ranks(dist, dt, args.steps * len(run.items))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": world * args.steps * len(run.items) / dt, "unit": "utt/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": dt / args.steps * 1e3, "per_rank_utt_s": per, "stub": True}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("single", "batch64", "mixed100"), default="single")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--vits-lanes", type=int, default=0,
                    help="batched workloads: concurrent vocoder streams (0 = the engine default)")
    ap.add_argument("--vocoder-cus", type=int, default=64,
                    help="single workload: CUs reserved for the overlapped vocoder (0 = sequential)")
    ap.add_argument("--decode-cus", type=int, default=0,
                    help="single workload: CUs of the decode (0 = all but the vocoder's)")
    ap.add_argument("--decode-cu-offset", type=int, default=0,
                    help="single workload: first decode CU past the vocoder CUs")
    ap.add_argument("--streams-per-gpu", type=int, default=1,
                    help="single workload under torchrun: S ranks share one GPU, each decoding on "
                         "--decode-cus CUs of its own (offset rank %% S x decode-cus) beside the shared vocoder CUs")
    ap.add_argument("--concurrent-streams", type=int, default=2,
                    help="single workload, N=1: also time this many sentence streams sharing the GPU "
                         "(child ranks, --streams-per-gpu) and report them beside the headline (0/1 = off)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="batched workloads: 1 = each batch's vocoder beside the next batch's T2S, "
                         "0 = one batch at a time")
    ap.add_argument("--batch-vocoder-cus", type=int, default=0,
                    help="batched workloads: CUs of the vocoder lanes (the T2S gets the rest; 0 = shared)")
    ap.add_argument("--vocoder-first", action="store_true",
                    help="batched workloads: each decode waits for the previous batch's vocoder (no vocoder kernel "
                         "pending behind the persistent decode)")
    ap.add_argument("--lanes-all-cus", action="store_true",
                    help="with --batch-vocoder-cus: the vocoder lanes on every CU (the T2S stream keeps the split)")
    ap.add_argument("--lane-priority", type=int, default=None,
                    help="batched workloads: HIP stream priority of the vocoder lanes (lower = first)")
    ap.add_argument("--t2s-priority", type=int, default=None,
                    help="batched workloads: HIP stream priority of the engine (T2S) stream")
    ap.add_argument("--shard", type=str, default="",
                    help="mixed100 on one GPU: run only LPT shard R of an N-rank job (R/N), to time "
                         "one rank of an N-GPU run (tools/shard_projection.py)")
    ap.add_argument("--stub-ms", type=float, default=0.0,
                    help=argparse.SUPPRESS)   # tests: a CPU stub replica whose step sleeps this long
    args = ap.parse_args()

    if args.shard and args.workload != "mixed100":
        ap.error("--shard applies to --workload mixed100 (the LPT-sharded set)")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.stub_ms > 0:
        return stub_main(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    sub = local % args.streams_per_gpu          # stream index on this GPU
    local //= args.streams_per_gpu              # the GPU
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")      # host group: barrier + max time only (no RCCL)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    # a non-default stream: work on the legacy null stream would serialise with every
    # blocking stream (the CU-masked engine streams are blocking)
    torch.cuda.set_stream(torch.cuda.Stream(dev))

    from genie_tts_amd import workloads, replicas
    from genie_tts_amd.probe import persist_roofline, composite_roofline
    wl = {"single": workloads.single, "batch64": workloads.batch64, "mixed100": workloads.mixed100}[args.workload]()
    if args.workload == "mixed100":
        reqs = [replicas.Request(i, it.text_seq, it.text_bert, it.force_steps, it.bert_ids, it.word2ph)
                for i, it in enumerate(wl.items)]
        if args.shard:
            if world > 1:
                raise SystemExit("--shard is a one-process measurement of one rank's shard")
            sr, sn = (int(x) for x in args.shard.split("/"))
            shard = replicas.lpt_assign([replicas.predicted_cost(r) for r in reqs], sn)[sr]
        else:
            shard = replicas.lpt_assign([replicas.predicted_cost(r) for r in reqs], world)[rank]
        items = [wl.items[i] for i in shard]
        # the whole set per step, over all ranks (a --shard run: its own sentences only)
        units_per_step = len(items) if args.shard else len(wl.items)
    else:
        items = wl.items
        units_per_step = world * len(items)       # every replica runs the workload (weak scaling)
    run = Runner(wl, items, dev, local if world > 1 else 0)
    if args.vits_lanes:
        run.eng.set_option("vits_lanes", args.vits_lanes)
    if args.batch_vocoder_cus and args.workload != "single":
        run.eng.set_vocoder_cus(args.batch_vocoder_cus)
    if args.vocoder_first:
        run.eng.set_option("vocoder_first", 1)
    if args.lanes_all_cus:
        run.eng.set_option("lanes_all_cus", 1)
    if args.lane_priority is not None:
        run.eng.set_option("lane_priority", args.lane_priority)
    if args.t2s_priority is not None:
        run.eng.set_option("t2s_priority", args.t2s_priority)
    timed_single = args.workload == "single"
    run.eng.set_timing(True)                      # phase events (+ live dominant-kernel events at B = 1)
    overlap = timed_single and args.vocoder_cus > 0
    pipelined = not timed_single and args.pipeline > 0
    step = run.step_pipelined if pipelined else run.step
    if overlap:
        run.eng.set_option("decode_cus", args.decode_cus)
        run.eng.set_option("decode_cu_offset", args.decode_cu_offset + sub * args.decode_cus)
        run.eng.set_vocoder_cus(args.vocoder_cus)
        sems, n_samples = run.stream(max(1, args.warmup))
    else:
        for _ in range(args.warmup):
            sems, n_samples = step()
        run.drain()
    torch.cuda.synchronize()
    run.phase = {k: 0.0 for k in run.phase}
    if timed_single:
        run.eng.set_timing(True)                  # reset live-kernel samples: only the timed region counts

    phase_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if overlap:   # the whole stream, fill and drain included (the last vocoder too)
        sems, n_samples = run.stream(args.steps, phase_ms)
    else:   # pipelined: the fill (first T2S alone) and the drain (last vocoder alone) are timed
        for _ in range(args.steps):
            sems, n_samples = step()
            if timed_single:
                phase_ms.append(run.eng.timing())
        run.drain()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    dt, per_rank = over_ranks(dist, dt, args.steps * len(items))   # this rank's utterances

    R_, H_ = wl.reference.ref_seq.shape[1], wl.reference.ssl.shape[2]
    n0s = [R_ + it.text_seq.shape[1] + H_ // 2 for it in items]
    roof = persist_roofline(run.eng, n0=n0s[0], steps=items[0].force_steps, B=1) if timed_single else None
    seq = None
    if overlap and rank == 0 and world == 1:
        # one utterance alone (no overlap, every CU): the single-request latency
        run.eng.set_vocoder_cus(0)
        run.step()
        torch.cuda.synchronize()
        ns = min(args.steps, 10)
        ts = time.perf_counter()
        for _ in range(ns):
            run.step()
        torch.cuda.synchronize()
        seq = (time.perf_counter() - ts) / ns

    ms_per_step = dt / args.steps * 1e3
    utt_s = units_per_step * args.steps / dt
    audio_s = n_samples / SR                                  # this rank's audio per step
    rtf = (dt / args.steps) / audio_s
    tokens = [int(s.size) for s in sems]

    out = {
        "metric": METRIC,
        "value": utt_s,
        "unit": "utt/s",
        "n_gpus": world // args.streams_per_gpu,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.workload == "mixed100" else "weak",
        "vs_baseline": None,
        "dtype": "f32 activations (fp16-valued weights; split-fp16 MFMA GEMMs)",
        "data": "synthetic (seeded inputs, synthetic fp16-valued weights; no checkpoints offline)",
        "rtf": rtf,
        "x_realtime": 1.0 / rtf,
        "audio_s_per_step": audio_s,
        "tokens_per_step": sum(tokens),
        "per_rank_utt_s": per_rank,
    }
    if args.workload == "single":
        it = items[0]
        out["config"] = {"workload": "configs[1]: V2 speaker, single utterance, greedy, 1 utt per replica" +
                                     (f"; a stream of such utterances, each one's vocoder on {args.vocoder_cus} CUs "
                                      "beside the next one's T2S" if overlap else ""),
                         "ref_phones": R_, "text_phones": it.text_seq.shape[1], "ssl_frames": H_,
                         "loop_steps": it.force_steps, "semantic_tokens": tokens[0],
                         "samples": n_samples, "parallelism": f"replicas x{world}",
                         "vocoder_cus": args.vocoder_cus,
                         "streams_per_gpu": args.streams_per_gpu,
                         "decode_cus": args.decode_cus or None,
                         "persist_timeouts": run.eng.counter("persist_timeouts"),
                         "vits_f32_reruns": run.eng.counter("vits_f32_reruns")}
        if roof is not None and "achieved" in roof and rank == 0:
            # the achievable HBM rate beside the spec peak -- a grid-stride device
            # copy of 1 GiB (gsv_debug_hbm_copy; read + write bytes), outside the timed region
            from genie_tts_amd.engine import hbm_copy_ms
            src = torch.empty(1 << 28, dtype=torch.float32, device=dev)
            dst = torch.empty_like(src)
            ach = 2 * src.numel() * 4 / (hbm_copy_ms(src, dst, 10) * 1e-3) / 1e9
            del src, dst
            roof["achievable_hbm"] = {"value": ach, "unit": "GB/s", "frac": roof["achieved"] / ach,
                                      "how": "non-temporal grid-stride copy of 1 GiB x 10 on this GPU "
                                             "(gsv_debug_hbm_copy), read + write bytes"}
        out["roofline"] = roof
        if seq is not None:
            out["sequential"] = {"utt_s": 1.0 / seq, "ms_per_utt": seq * 1e3, "x_realtime": audio_s / seq,
                                 "note": "one utterance at a time on every CU (single-request latency)"}
        if phase_ms:
            pm = np.mean(np.asarray(phase_ms), axis=0)
            out["phase_ms"] = {"encode": float(pm[0]), "prefill": float(pm[1]), "decode": float(pm[2]),
                               "vits": float(pm[3])}
            out["roofline_utterance"] = composite_roofline(
                ms_per_step, n0s, [it.force_steps], tokens, wl.version,
                {"decode": float(pm[2]), "prefill": float(pm[1]), "vits": float(pm[3])})
    else:
        out["config"] = {"workload": wl.name + (" (top-k %d sampled)" % wl.top_k if not wl.greedy else " (greedy)"),
                         "version": wl.version, "sentences": len(wl.items), "sentences_this_rank": len(items),
                         "text_phones": [int(i.text_seq.shape[1]) for i in items][:8] + ["..."],
                         "semantic_tokens_this_rank": sum(tokens), "parallelism": f"replicas x{world}" +
                         (" (LPT shards)" if args.workload == "mixed100" else ""),
                         "pipelined": pipelined,
                         "vits_f32_reruns": run.eng.counter("vits_f32_reruns")}
        if args.shard:
            out["config"]["shard"] = args.shard
        ph = {k: v / args.steps * 1e3 for k, v in run.phase.items()}
        out["phase_ms"] = ph
        out["roofline_utterance"] = composite_roofline(ms_per_step, n0s, [it.force_steps for it in items], tokens,
                                                       wl.version)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "single":
        # every CPU this job is allotted: the GPU box gives one GPU's job 16 host CPUs
        # (OMP_NUM_THREADS=16 there) although the machine shows more; here: all 8
        threads = min(int(os.environ.get("OMP_NUM_THREADS") or 10 ** 6), len(os.sched_getaffinity(0)))
        cdt, cs = cpu_baseline(wl, threads)
        model = ""
        try:
            with open("/proc/cpuinfo") as f:
                model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
        except Exception:
            pass
        out["cpu_baseline"] = {"value": 1.0 / cdt, "unit": "utt/s", "cores": threads, "kind": "port",
                               "cores_note": "min(OMP_NUM_THREADS, len(sched_getaffinity(0))): the job's CPU share on the GPU box",
                               "sample": f"1 full utterance ({cs} samples) of the same workload, "
                                         f"oracle/restate.py torch-fp32 on {model}",
                               "rtf": cdt / (cs / SR)}
    if (rank == 0 and world == 1 and overlap and args.concurrent_streams > 1 and args.streams_per_gpu == 1):
        out["concurrent_streams"] = concurrent_streams(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    run.eng.close()


if __name__ == "__main__":
    main()
