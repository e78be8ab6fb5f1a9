#!/bin/bash
# Round-4 GPU session Y: k_fused4 workgroup order (band fastest) -- traffic and time.
set -o pipefail
OUT=gpurun_out/r04y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/traffic_ab.py $OUT 32 base ord1 ord1r42 ord1r18 2>&1 | tee $OUT/traffic.txt || exit 1
timeout -k 10 500 python tools/ab_fused.py 16 base ord1 ord1r42 ord1r18 base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
