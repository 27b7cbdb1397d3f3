#!/bin/bash
# Debug build of the persistent decode kernels (-DPERSIST_DBG dump points) as an
# alternative library genie_tts_amd/_lib/alt_dbg/libgenie_engine.so (GENIE_ENGINE_LIB);
# the other objects come from the in-tree build.
set -e
OUT=genie_tts_amd/_lib/alt_dbg
mkdir -p $OUT
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics -Xclang -target-feature -Xclang -packed-fp32-ops -DPERSIST_DBG"
for s in t2s_persist1 t2s_persist1m t2s_persistm; do
  /opt/rocm/bin/hipcc $F -Igenie_tts_amd/csrc -c genie_tts_amd/csrc/$s.hip -o $OUT/$s.o
done
OBJS=$(ls genie_tts_amd/_lib/obj/*.o | grep -v "/t2s_persist1.hip.o\|/t2s_persist1m.hip.o\|/t2s_persistm.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgenie_engine.so $OBJS $OUT/t2s_persist1.o $OUT/t2s_persist1m.o $OUT/t2s_persistm.o
echo $OUT/libgenie_engine.so
