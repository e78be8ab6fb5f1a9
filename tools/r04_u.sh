#!/bin/bash
# Round-4 GPU session U: four-column kernel with 29 weight pairs in SGPRs -> 124 VGPRs and
# 4 waves per SIMD at 1 row of prefetch (A/B).
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 500 python tools/ab_fused.py 16 base w29 w29p1e4 w29p2e4 w29p1e4r42 w29p1e4r24 base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
