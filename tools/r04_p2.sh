#!/bin/bash
# Round-4 GPU session P2: A/B of the bank-conflict-free weight layout in the bf16 MFMA conv.
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 200 python tools/ab_ops.py wide 10 base cvold base%HYGRID_CONV_DMA=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide.txt
