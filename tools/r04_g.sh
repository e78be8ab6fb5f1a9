#!/bin/bash
# Round-4 GPU session G: line-aligned triangle-kernel windows and the LDS-DMA-staged wide
# conv -- parity first, then A/Bs and counters.
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_hexdown.py tests/test_gpu_down.py tests/test_gpu_conv_mfma.py > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_ops.py wide 8 base base%HYGRID_CONV_DMA=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide.txt
for op in hr0 hr1 hr2 up; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base u2 i0 base%HYGRID_DOWN=0 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab_ops.txt
timeout -k 10 200 python tools/ab_ops.py rt 8 rtv0 rtpd4 rtpd2 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_rt.txt
bash tools/pmc_kernel.sh r04g/pmc_tri_hr0 k_hexresize_down -- python3 tools/prof_ops.py hr0 3 > $OUT/pmc_tri_hr0.log 2>&1 || { tail -5 $OUT/pmc_tri_hr0.log; exit 1; }
bash tools/pmc_kernel.sh r04g/pmc_tri_up k_hexresize_down -- python3 tools/prof_ops.py up 3 > $OUT/pmc_tri_up.log 2>&1 || { tail -5 $OUT/pmc_tri_up.log; exit 1; }
grep -E "FETCH|WRITE|BANK|LDS_IDX|WAIT|WAVE_CYCLES|VMEM|ACTIVE_INST_ANY" $OUT/pmc_tri_hr0.log $OUT/pmc_tri_up.log
