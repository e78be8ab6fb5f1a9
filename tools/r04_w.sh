#!/bin/bash
# Round-4 GPU session W: k_fused4 band length at 4 waves per SIMD (fewer halo-row re-reads vs
# fewer, longer work units).
set -o pipefail
OUT=gpurun_out/r04w; mkdir -p $OUT
timeout -k 10 500 python tools/ab_fused.py 16 base rb30 rb60 rb84 rb126 base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
