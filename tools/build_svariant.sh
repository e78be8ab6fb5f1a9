#!/bin/bash
# Build a tuning variant of the whole libhygrid_hip.so with ONE source recompiled under
# extra -D flags (Makefile flags; -fno-slp-vectorize for the streaming sources), linked with
# the other objects of the last `make`.  Time it with tools/ab_ops.py / tools/ab_fused.py.
#   tools/build_svariant.sh NAME SRC.hip -DST_RB_=64 [-D...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
NAME=$1; SRC=$2; shift 2
BASE=$(basename "$SRC" .hip)
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
EXTRA=""
case "$BASE" in fused|fused_conv|resample_stream|pyramid_fused|pyramid_stream) EXTRA="-fno-slp-vectorize" ;; esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $EXTRA "$@" \
    -I"$PKG/csrc" -c "$PKG/csrc/$BASE.hip" -o "$OBJ/variants/${BASE}_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" \
    $(ls "$OBJ"/*.o | grep -v "/$BASE.o\$") "$OBJ/variants/${BASE}_$NAME.o"
echo "$OUT/libhygrid_$NAME.so"
