#!/bin/bash
# Round-4 GPU session K: what limits the upsampling triangle kernel (tri_up.hip) -- no-store /
# no-load diagnostics, prefetch depth, unit order, plane chunks.
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
export TMPDIR=/tmp
for op in up upn; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base nost nold pd2 ord1 base%HYGRID_TU_CHUNKS=4 base%HYGRID_TU_CHUNKS=16 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.txt || exit 1
done
