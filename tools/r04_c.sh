#!/bin/bash
# Round-4 GPU session C: triangle-kernel depth / rows / occupancy variants, MD 2 prefetch
# depth, then counters of the triangle kernel and of the general kernel it replaces.
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
for op in hr0 hr1 hr2 up; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 t0 tp2 trb4 tw2 tp2w2 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
[ -f hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd/HyGrid/_lib/variants/libhygrid_rtpd2.so ] && { timeout -k 10 200 python tools/ab_ops.py rt 8 rtv0 rtpd4 rtpd2 >> $OUT/ab_ops.txt 2>&1 || exit 1; }
grep -v amdgpu.ids $OUT/ab_ops.txt
for op in hr0 hr2 up; do
  bash tools/pmc_kernel.sh r04c/pmc_tri_$op k_hexresize_down -- python3 tools/prof_ops.py $op 3 > $OUT/pmc_tri_$op.log 2>&1 || { tail -5 $OUT/pmc_tri_$op.log; exit 1; }
done
export HYGRID_DOWN=0
for op in hr0 hr1 hr2; do
  bash tools/pmc_kernel.sh r04c/pmc_lds_$op k_resample_lds -- python3 tools/prof_ops.py $op 3 > $OUT/pmc_lds_$op.log 2>&1 || { tail -5 $OUT/pmc_lds_$op.log; exit 1; }
done
tail -n 25 $OUT/pmc_tri_hr0.log $OUT/pmc_tri_up.log
