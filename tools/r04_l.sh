#!/bin/bash
# Round-4 GPU session L: the upsampling kernel's compute floor (no loads, no stores).
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
export TMPDIR=/tmp
for op in up upn; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base none nost nold 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.txt || exit 1
done
