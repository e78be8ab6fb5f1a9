#!/bin/bash
# Round-4 GPU session AA: upsampling kernel with VGPR-staged row loads (TU_VLD) vs LDS-DMA.
set -o pipefail
OUT=gpurun_out/r04aa; mkdir -p $OUT
for op in up upn; do
  timeout -k 10 200 python tools/ab_ops.py $op 10 base vld vld2 vld4 vld5 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.txt || exit 1
done
