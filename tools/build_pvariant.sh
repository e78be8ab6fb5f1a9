#!/bin/bash
# Build a tuning variant of libhygrid_hip.so with pyramid_fused.hip recompiled under extra -D
# flags, linked with the pyramid objects of the last `make` (hg_hex_pyramid_level and what it
# dispatches to).  Run it with tools/ab_ops.py pyr* <name>.
#   tools/build_pvariant.sh NAME -DFU_DMA=2 [-D...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
NAME=$1; shift
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize "$@" \
    -I"$PKG/csrc" -c "$PKG/csrc/pyramid_fused.hip" -o "$OBJ/variants/pyramid_fused_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" \
    "$OBJ/abi.o" "$OBJ/pyramid.o" "$OBJ/pyramid_stream.o" "$OBJ/variants/pyramid_fused_$NAME.o"
echo "$OUT/libhygrid_$NAME.so"
