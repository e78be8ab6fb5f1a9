#!/bin/bash
# Round-4 GPU session B: the wide-piece triangle kernel (parity + A/B against the general
# kernel), then the pyramid / fused variant A/Bs and the secondary lines' counters.
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_hexdown.py tests/test_gpu_down.py > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for op in hr0 hr1 hr2 up; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base base%HYGRID_TSK_UPW=4 base%HYGRID_DOWN=0 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
cat $OUT/ab_ops.txt
for op in pyrfr pyr1 pyr2; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 p0 pdma pdma2 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/ab_fused.py 8 v0 v05 dmans dmans5 dmans6 > $OUT/ab_fused.txt 2>&1 || exit 1
cat $OUT/ab_ops.txt $OUT/ab_fused.txt
for op in rt pyr0; do
  bash tools/pmc_kernel.sh r04b/pmc_$op k_fused -- python3 tools/prof_ops.py $op 3 > $OUT/pmc_$op.log 2>&1 || { tail -5 $OUT/pmc_$op.log; exit 1; }
done
tail -30 $OUT/pmc_rt.log $OUT/pmc_pyr0.log
