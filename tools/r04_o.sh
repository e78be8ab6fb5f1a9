#!/bin/bash
# Round-4 GPU session O: counters of the LDS-DMA-staged wide bf16 conv (k_hexconv_mfma_bf16d)
# + the downsampling kernel's parity after the record-scheduling change.
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_hexdown.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_kernel.sh r04o/pmc_wide k_hexconv_mfma_bf16d -- python3 tools/prof_ops.py wide 3 > $OUT/pmc_wide.log 2>&1 || { tail -5 $OUT/pmc_wide.log; exit 1; }
cat gpurun_out/r04o/pmc_wide/summary.txt
