#!/bin/bash
# Round-4 GPU session S: four-column kernel band length / prefetch variants (in-process A/B).
set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT
timeout -k 10 400 python tools/ab_fused.py 10 base f4rb24 f4rb18 f4rb30 f4rb60 f4pd2 f4pd4 base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
