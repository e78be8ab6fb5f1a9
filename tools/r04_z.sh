#!/bin/bash
# Round-4 GPU session Z: single-buffered weight chunks in the bf16 MFMA conv (3 workgroups per
# CU) -- parity, then A/B against double-buffered and register-staged.
set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_conv_mfma.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_ops.py wide 12 base base%HYGRID_CONV_WDB=1 base%HYGRID_CONV_DMA=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide.txt
