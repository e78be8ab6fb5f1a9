#!/bin/bash
# Build a variant of the whole libhygrid_hip.so in which the named kernel sources are compiled
# from git revision REV (the csrc tree of that commit, headers included) and every other object
# is the last `make`'s: an in-process A/B of a change against the code it replaced.
#   tools/build_revvariant.sh NAME REV SRC.hip [SRC.hip ...]   [-- extra -D flags]
#       -> HyGrid/_lib/variants/libhygrid_NAME.so   (run with tools/ab_*.py ... NAME)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKGREL=hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd
PKG=$ROOT/$PKGREL
NAME=$1; REV=$2; shift 2
SRCS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SRCS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
OBJ=$PKG/build/obj
OUT=$PKG/HyGrid/_lib/variants
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$OUT" "$OBJ/variants" "$TMP/csrc" "$TMP/include"
git -C "$ROOT" archive "$REV" "$PKGREL/csrc" include | tar -x -C "$TMP"
skip=()
for s in "${SRCS[@]}"; do
    base=$(basename "$s" .hip)
    slp=""; case "$base" in fused|fused4|fused_conv|resample_stream|pyramid_fused|pyramid_stream) slp=-fno-slp-vectorize ;; esac
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $slp "$@" \
        -I"$TMP/$PKGREL/csrc" -c "$TMP/$PKGREL/csrc/$base.hip" -o "$OBJ/variants/${base}_$NAME.o"
    skip+=("$base")
done
objs=()
for o in $(cd "$OBJ" && ls *.o | sed 's/\.o$//'); do
    if printf '%s\n' "${skip[@]}" | grep -qx "$o"; then objs+=("$OBJ/variants/${o}_$NAME.o"); else objs+=("$OBJ/$o.o"); fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libhygrid_$NAME.so" "${objs[@]}"
echo "$OUT/libhygrid_$NAME.so"
