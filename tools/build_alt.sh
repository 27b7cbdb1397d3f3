#!/bin/bash
# Build an alternative libgenie_engine.so in which ONE source is replaced (A/B of a
# kernel variant on the GPU box via GENIE_ENGINE_LIB).  The other objects come from
# the in-tree build.
# Usage: bash tools/build_alt.sh NAME REPLACED_SOURCE.hip VARIANT_SOURCE.hip
set -e
NAME=$1; SRC=$2; VAR=$3
OUT=genie_tts_amd/_lib/alt_$NAME
mkdir -p $OUT
cp "$VAR" genie_tts_amd/csrc/_alt_variant.hip
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics -Xclang -target-feature -Xclang -packed-fp32-ops -DGSV_NO_PACKED_FP32=1 \
  -c genie_tts_amd/csrc/_alt_variant.hip -o $OUT/variant.o
rm -f genie_tts_amd/csrc/_alt_variant.hip
OBJS=$(ls genie_tts_amd/_lib/obj/*.o | grep -v "/$(basename $SRC).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgenie_engine.so $OBJS $OUT/variant.o
echo $OUT/libgenie_engine.so
