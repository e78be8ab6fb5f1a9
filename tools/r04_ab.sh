#!/bin/bash
# Round-4 GPU session AB: parity of the VGPR-staged upsampling kernel (default now).
set -o pipefail
OUT=gpurun_out/r04ab; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_triup.py tests/test_gpu_hexdown.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
exit $rc
