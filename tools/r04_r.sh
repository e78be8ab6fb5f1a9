#!/bin/bash
# Round-4 GPU session R: the four-column headline kernel (fused4.hip) -- parity, then A/B
# against the two-column kernel, then its counters.
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_fused4.py tests/test_gpu_pipeline.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_fused.py 10 base base%HYGRID_FUSED4=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
