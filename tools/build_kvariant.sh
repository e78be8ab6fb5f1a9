#!/bin/bash
# Build a tuning variant of libhygrid_hip.so with ONE kernel source recompiled under extra -D
# flags, linked with the objects of the last `make` that the fused entry points need (abi,
# pipeline, fused, fused4, rt4: what tools/ab_fused.py and tools/ab_ops.py rt call).
#   tools/build_kvariant.sh fused4.hip NAME -DF4_RB_=60 [-D...]
#       -> HyGrid/_lib/variants/libhygrid_NAME.so   (run with tools/ab_*.py ... NAME)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
SRC=$1; NAME=$2; shift 2
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
base=$(basename "$SRC" .hip)
# SLP=1: keep the SLP vectoriser (the Makefile's default for most objects)
slp=-fno-slp-vectorize; [ "${SLP:-0}" = 1 ] && slp=
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $slp "$@" \
    -I"$PKG/csrc" -c "$PKG/csrc/$SRC" -o "$OBJ/variants/${base}_$NAME.o"
objs=()
# FULL=1: every object of the library (for entry points outside the fused pipeline, e.g. the conv)
list="abi pipeline fused fused4"
[ "${FULL:-0}" = 1 ] && list=$(cd "$OBJ" && ls *.o | sed 's/\.o$//')
for o in $list; do
    if [ "$o" = "$base" ]; then objs+=("$OBJ/variants/${base}_$NAME.o"); else objs+=("$OBJ/$o.o"); fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" "${objs[@]}"
echo "$OUT/libhygrid_$NAME.so"
