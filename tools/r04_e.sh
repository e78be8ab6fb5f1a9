#!/bin/bash
# Round-4 GPU session E: does line alignment of the triangle kernel's output windows matter?
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
for op in hr0 up hr1; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 i0 i0%HYGRID_TSK_NOUT=192 i0%HYGRID_TSK_NOUT=188 i0%HYGRID_TSK_NOUT=128 i0%HYGRID_TSK_NOUT=124 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab_ops.txt
[ -f hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd/HyGrid/_lib/variants/libhygrid_rtpd2.so ] && { timeout -k 10 200 python tools/ab_ops.py rt 8 rtv0 rtpd4 rtpd2 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_rt.txt; }
exit 0
