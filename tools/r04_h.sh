#!/bin/bash
# Round-4 GPU session H (re-entry): full GPU suite + smoke + default bench line on the current
# tree, then session G's A/Bs and counters (triangle kernel, LDS-DMA wide conv).
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 200 python tools/ab_ops.py wide 8 base base%HYGRID_CONV_DMA=0 2>&1 | grep -v amdgpu.ids | tee $OUT/ab_wide.txt
for op in hr0 hr1 hr2 up; do
  timeout -k 10 200 python tools/ab_ops.py $op 8 base base%HYGRID_DOWN=0 >> $OUT/ab_ops.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/ab_ops.txt
timeout -k 10 120 ./tools/microbench/walk6 > $OUT/walk6.txt 2>&1 || { tail $OUT/walk6.txt; exit 1; }
cat $OUT/walk6.txt
