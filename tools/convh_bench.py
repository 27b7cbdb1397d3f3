"""Microbenchmark of the f16-split MRF conv (vits_convh.hip) on the generator's
stage shapes: per (C, T, k, dil) the kernel time for each tile config
(GENIE_CONVH_CFG) and debug mode (GENIE_CONVH_DBG: 1 no MFMA, 2 no global loads).
Each configuration runs in its own subprocess (the env knobs are read once)."""
import json
import os
import subprocess
import sys

SHAPES = [(256, 1600, 11, 5), (256, 1600, 3, 1), (128, 12800, 11, 5), (128, 12800, 3, 1),
          (64, 25600, 11, 5), (32, 51200, 11, 5), (16, 102400, 11, 5)]

CHILD = r'''
import sys, json, torch
sys.path.insert(0, ".")
import ctypes
from genie_tts_amd.engine import lib, _stream
L = lib()
P = lambda t: ctypes.c_void_p(t.data_ptr())
res = []
for c, T, k, d in SHAPES:
    x = torch.randn(c, T, device="cuda")
    v = (torch.randn(c, c, k) / (c * k) ** 0.5).half().float()
    wh = v.half().permute(0, 2, 1).contiguous().cuda()
    sc = torch.ones(c, device="cuda")
    b = torch.zeros(c, device="cuda")
    pad = d * (k - 1) // 2
    out = torch.empty(c, T, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = _stream()
    def run():
        rc = L.gsv_debug_conv1d_h(P(x), c, T, P(wh), P(sc), c, k, d, pad, P(b), P(out), T, 1,
                                  ctypes.c_float(0.1), P(ovf), st)
        assert rc == 0
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        run()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    res.append((c, T, k, d, us, 2.0 * c * c * k * T / us / 1e6))
print(json.dumps(res))
'''

def main():
    if "--inproc" in sys.argv:      # one process, env already set (for rocprofv3 --kernel-trace)
        exec(f"SHAPES={SHAPES!r}\n" + CHILD, {"__name__": "__child__"})
        return
    out = {}
    for cfg in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["-1", "0", "1", "2", "3"]):
        for dbg in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0"]):
            env = dict(os.environ, GENIE_CONVH_CFG=cfg, GENIE_CONVH_DBG=dbg)
            r = subprocess.run([sys.executable, "-c", f"SHAPES={SHAPES!r}\n" + CHILD], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(cfg, dbg, "FAILED", r.stderr[-2000:]); sys.exit(1)
            res = json.loads(r.stdout.strip().splitlines()[-1])
            for c, T, k, d, us, tf in res:
                print(f"cfg {cfg:>2} dbg {dbg} C={c:4d} T={T:6d} k={k:2d} d={d}: {us:8.1f} us {tf:7.1f} TF/s ", flush=True)

main()
