"""CPU: the built library's gfx950 code holds no packed-FP32 VALU instruction.

On gfx950 a packed-FP32 op whose low result reads the high half of a source register pair
through op_sel (e.g. `v_pk_mul_f32 v[40:41], v[40:41], v[4:5] op_sel:[0,1]
op_sel_hi:[1,0]`) returned 0 in lanes 48-63 while MFMA-heavy waves ran on the same chip.
hipcc formed exactly that instruction in k_conv_h<1,32,1,1,4> (the polyphase ConvTranspose
input scale), and concurrent vocoder lanes then corrupted 1-2 frame windows (the r04
nondeterminism).  tools/pk_opsel_probe.hip reproduces the fault outside the engine:
op_sel'd forms fail beside MFMA streams, the plain form and the quiet chip do not
(profiles/r05_convt_race.txt).  The build turns the packed-fp32-ops target feature off
(genie_tts_amd/build.py); this test disassembles the library to check that it stays off.
"""
import os
import re
import shutil
import subprocess

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "genie_tts_amd", "_lib",
                   "libgenie_engine.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PACKED32 = re.compile(r"\bv_pk_(add|mul|fma|mov)_(f32|b32)\b")


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump absent")
def test_no_packed_fp32_ops_in_device_code(tmp_path):
    from genie_tts_amd import build as B
    assert "-packed-fp32-ops" in B.FLAGS
    B.build()                        # up to date (a no-op) or rebuilt with the current flags
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    # --offloading extracts each offload bundle next to its input file
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path)
    bundles = sorted(p for p in os.listdir(tmp_path) if p.endswith("gfx950"))
    assert bundles, "no gfx950 code object in the library"
    n_inst = 0
    for b in bundles:
        dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(tmp_path / b)], check=True, capture_output=True,
                             text=True).stdout
        bad = [l.strip() for l in dis.splitlines() if PACKED32.search(l)]
        assert not bad, f"{b}: {len(bad)} packed-FP32 instructions, e.g. {bad[:3]}"
        n_inst += dis.count("\n")
    assert n_inst > 100_000          # the disassembly really covered the kernels


def test_library_marks_its_build_and_the_loader_checks_it():
    """The build defines GSV_NO_PACKED_FP32 with the target-feature flag; gsv_version reports it,
    and engine.lib() refuses a library without the mark (build.py)."""
    import ctypes
    from genie_tts_amd import build as B
    assert "-DGSV_NO_PACKED_FP32=1" in B.FLAGS
    B.build()
    L = ctypes.CDLL(LIB)
    L.gsv_version.restype = ctypes.c_char_p
    assert b"no packed-fp32" in L.gsv_version()
