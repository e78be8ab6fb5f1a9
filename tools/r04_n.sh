#!/bin/bash
# Round-4 GPU session N: upsampling kernel band / width variants (A/B).
set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT
export TMPDIR=/tmp
for op in up upn; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base rb4 rb4k k2 rb6 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.txt || exit 1
done
