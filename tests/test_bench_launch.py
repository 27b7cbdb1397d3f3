"""CPU: `python bench.py --gpus N` without a launcher starts N ranks itself
(torch.distributed.run child, before any GPU call) and prints rank 0's JSON line with
n_gpus = N, the max-over-ranks time and per-rank rates.  Stub replicas (--stub-ms)
replace the engine; the GPU path shares the launcher and the reduction (bench.py)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_launches_n_ranks():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--warmup", "1", "--stub-ms", "20"], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["stub"] and len(d["per_rank_utt_s"]) == 2
    # rank 1 steps 1.5x slower: the job's time is the slowest rank's
    assert d["ms_per_step"] >= 29.0, d
    assert abs(d["value"] - 2 * 4 / (d["ms_per_step"] * 4e-3)) < 1e-6 * d["value"]
    assert d["per_rank_utt_s"][0] > d["per_rank_utt_s"][1]
