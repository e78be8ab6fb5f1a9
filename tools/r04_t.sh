#!/bin/bash
# Round-4 GPU session T: four-column kernel, second box: band 30 / 36, prefetch 2 (A/B).
set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
timeout -k 10 400 python tools/ab_fused.py 16 base f4rb30 f4rb36 f4pd2 f4rb30pd2 base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
