#!/bin/bash
# Build a tuning variant of libhygrid_hip.so with fused.hip recompiled under extra -D
# flags, linked with the objects of the last `make`.  Run it with HYGRID_LIB=<path>.
#   tools/build_fvariant.sh NAME -DFU_PD=2 [-D...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
NAME=$1; shift
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -DFU_MIN_INST=${FU_MIN_INST:-1} "$@" \
    -I"$PKG/csrc" -c "${FUSED_SRC:-$PKG/csrc/fused.hip}" -o "$OBJ/variants/fused_$NAME.o"
# slim library: only what hg_pipeline_r2h_conv_h2r needs (tools/ab_fused.py calls nothing else)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" \
    "$OBJ/abi.o" "$OBJ/pipeline.o" "$OBJ/variants/fused_$NAME.o"
echo "$OUT/libhygrid_$NAME.so"
