"""Build libgenie_engine.so (gfx950) in-tree with hipcc.

One shared library, no torch dependency: C ABI in include/genie_engine.h.
Objects are rebuilt when their source, a .hip it includes, or any header is newer, and all
of them when the compiler flags change (a hash of FLAGS is kept beside the objects).
"""
from __future__ import annotations

import glob
import hashlib
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIB_DIR, "libgenie_engine.so")
ARCH = os.environ.get("GENIE_OFFLOAD_ARCH", "gfx950")
# No packed-FP32 VALU ops (v_pk_{add,mul,fma,mov}_*32) in the device code.  On gfx950 a packed op
# whose LOW result reads the HIGH half of a source pair through op_sel (v_pk_mul_f32 d, a, b
# op_sel:[0,1]) returned 0 in lanes 48-63 while MFMA-heavy waves ran beside it: the vocoder's
# nondeterministic 1-2 frame errors of r04 (profiles/r05_convt_race.txt; tools/pk_opsel_probe.hip
# reproduces it outside the engine).  hipcc forms such ops from ordinary float pairs, so the
# feature is off for every kernel, and tests/test_isa_audit.py checks the built library.
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-DGSV_NO_PACKED_FP32=1"]
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-Wno-unused-value", "-munsafe-fp-atomics", *NO_PACKED_FP32]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def flags_hash() -> str:
    return hashlib.sha256(" ".join(FLAGS).encode()).hexdigest()[:16]


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(os.path.join(LIB_DIR, "obj"), exist_ok=True)
    # objects built with other flags (e.g. before NO_PACKED_FP32) are stale whatever their mtime
    stamp = os.path.join(LIB_DIR, "obj", "FLAGS")
    fh = flags_hash()
    if not os.path.exists(stamp) or open(stamp).read().strip() != fh:
        force = True
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdr = _headers_mtime()
    cc = _hipcc()

    def src_mtime(src):
        # a .hip that includes another .hip (t2s_persist1m.hip) is stale when the included one changes
        t = os.path.getmtime(src)
        with open(src) as f:
            for line in f:
                m = re.match(r'\s*#include\s+"([^"]+\.hip)"', line)
                if m:
                    t = max(t, os.path.getmtime(os.path.join(CSRC, m.group(1))))
        return t

    def compile_one(src):
        obj = os.path.join(LIB_DIR, "obj", os.path.basename(src) + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(src_mtime(src), hdr):
            return obj
        cmd = [cc, *FLAGS, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-6000:]}")
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    with open(stamp, "w") as f:
        f.write(fh + "\n")
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
