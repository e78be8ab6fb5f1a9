#!/bin/bash
# Round-4 GPU session Z2: wide conv with 2 output-channel tiles per workgroup (4 waves per SIMD,
# 4 workgroups per CU with single-buffered weights) vs 4 tiles.
set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
timeout -k 10 300 python tools/ab_ops.py wide 12 base base%HYGRID_CONV_NT=2 base%HYGRID_CONV_WDB=1 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide_nt.txt
