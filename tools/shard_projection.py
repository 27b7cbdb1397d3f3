"""configs[3] strong scaling, projected from one GPU: time every rank's LPT shard of an
N-rank mixed100 job (bench.py --workload mixed100 --shard R/N, one fresh process per
shard, sequentially on this GPU) and report the job rate the N-GPU run would have, the
100 sentences over the slowest shard's time, beside the one-GPU rate.  Replicas share
nothing, so a rank's time on its own GPU is its shard's time here.
Usage: python tools/shard_projection.py [N ...]   (default 2 4 8); one JSON line"""
import json
import subprocess
import sys

ns = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
steps, warmup = 20, 3


def run(extra):
    cmd = [sys.executable, "bench.py", "--workload", "mixed100", "--no-cpu-baseline", "--steps", str(steps),
           "--warmup", str(warmup)] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


one = run([])
out = {"one_gpu": {"utt_s": one["value"], "ms_per_set": one["ms_per_step"]}, "projected": {}}
print(json.dumps({"n": 1, "ms_per_set": one["ms_per_step"]}), flush=True)
for n in ns:
    shards = []
    for r in range(n):
        d = run(["--shard", f"{r}/{n}"])
        shards.append({"rank": r, "sentences": d["config"]["sentences_this_rank"], "ms": d["ms_per_step"]})
        print(json.dumps({"n": n, **shards[-1]}), flush=True)
    slow = max(s["ms"] for s in shards)
    rate = 100.0 / (slow * 1e-3)
    out["projected"][str(n)] = {"utt_s": rate, "slowest_shard_ms": slow, "efficiency": rate / (n * one["value"]),
                                "shards": shards}
print(json.dumps(out), flush=True)
