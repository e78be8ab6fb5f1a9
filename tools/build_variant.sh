#!/bin/bash
# Build a tuning variant of libhygrid_hip.so: pipeline.hip recompiled with extra -D flags
# and linked with the objects of the last `make`.  Run a variant with HYGRID_LIB=<path>.
#   tools/build_variant.sh NAME -DPL_S_PD=3 [-D...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
NAME=$1; shift
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" \
    -c "$PKG/csrc/pipeline.hip" -o "$OBJ/variants/pipeline_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" \
    "$OBJ/abi.o" "$OBJ/resample.o" "$OBJ/hexconv.o" "$OBJ/conv_stream.o" "$OBJ/variants/pipeline_$NAME.o"
echo "$OUT/libhygrid_$NAME.so"
