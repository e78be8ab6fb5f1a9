#!/bin/bash
# Round-4 GPU session I: the upsampling triangle kernel (tri_up.hip) -- parity first, then
# A/B against the general kernels and the downsampling triangle kernel, then counters.
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_triup.py tests/test_gpu_hexdown.py > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_ops.py up 8 base base%HYGRID_UP=0 base%HYGRID_DOWN=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_up.txt
timeout -k 10 200 python tools/ab_ops.py upn 8 base base%HYGRID_UP=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_upn.txt
bash tools/pmc_kernel.sh r04i/pmc_up k_tri_up -- python3 tools/prof_ops.py up 3 > $OUT/pmc_up.log 2>&1 || { tail -5 $OUT/pmc_up.log; exit 1; }
grep -E "FETCH|WRITE|BANK|LDS_IDX|WAIT|WAVE_CYCLES|VMEM|VALU|ACTIVE_INST_ANY" $OUT/pmc_up.log
