#!/bin/bash
# Round-4 GPU session P: bank-conflict-free weight fragments in the bf16 MFMA conv -- parity,
# A/B against the previous layout, counters.
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_conv_mfma.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_ops.py wide 10 base cvold base%HYGRID_CONV_DMA=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide.txt
bash tools/pmc_kernel.sh r04p/pmc_wide k_hexconv_mfma_bf16d -- python3 tools/prof_ops.py wide 3 > $OUT/pmc_wide.log 2>&1 || { tail -5 $OUT/pmc_wide.log; exit 1; }
grep -E "BANK|IDX_ACTIVE|WAIT_ANY|WAVE_CYCLES|INSTS_LDS" gpurun_out/r04p/pmc_wide/summary.txt
