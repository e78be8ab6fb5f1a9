#!/bin/bash
# Round-4 GPU session D: interleaved lane ownership in the triangle kernel (parity + A/B).
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_hexdown.py tests/test_gpu_down.py > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for op in hr0 hr1 hr2 up; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 i0 iq2 iu1 ip2 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab_ops.txt
bash tools/pmc_kernel.sh r04d/pmc_tri_hr0 k_hexresize_down -- python3 tools/prof_ops.py hr0 3 > $OUT/pmc_tri_hr0.log 2>&1 || { tail -5 $OUT/pmc_tri_hr0.log; exit 1; }
grep -E "BANK|LDS_IDX|WAIT_ANY|WAVE_CYCLES|VMEM" $OUT/pmc_tri_hr0.log
[ -f hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd/HyGrid/_lib/variants/libhygrid_rtpd2.so ] && { timeout -k 10 200 python tools/ab_ops.py rt 8 rtv0 rtpd4 rtpd2 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_rt.txt; }
exit 0
