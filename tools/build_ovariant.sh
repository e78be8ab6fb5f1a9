#!/bin/bash
# Build a tuning variant of one kernel object (csrc/SRC.hip recompiled under extra -D flags)
# linked with the other objects of the last `make` into HyGrid/_lib/variants/libhygrid_NAME.so
# (slim: only the objects listed in OBJS, default the resampler entry points).  Run it with
# tools/ab_ops.py OP NAME ...
#   tools/build_ovariant.sh SRC NAME -DHD_PDP16=2 [-D...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
SRC=$1; NAME=$2; shift 2
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
mkdir -p "$OUT" "$OBJ/variants"
OBJS=${OBJS:-"abi resample resample_stream resample_down hexresize_down tri_up"}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" \
    -I"$PKG/csrc" -c "$PKG/csrc/$SRC.hip" -o "$OBJ/variants/${SRC}_$NAME.o"
LINK=""
for o in $OBJS; do
  if [ "$o" = "$SRC" ]; then LINK="$LINK $OBJ/variants/${SRC}_$NAME.o"; else LINK="$LINK $OBJ/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,--no-undefined -o "$OUT/libhygrid_$NAME.so" $LINK
echo "$OUT/libhygrid_$NAME.so"
