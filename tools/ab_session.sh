#!/bin/bash
# One GPU call: pyramid parity tests + tuning A/Bs (tools/ab_ops.py) -> gpurun_out/$1/
set -o pipefail
TAG=${1:-ab}; mkdir -p gpurun_out/$TAG; O=gpurun_out/$TAG/ab.txt; : > $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pyramid.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest_pyr.log 2>&1 || { echo "pyramid tests failed"; tail -30 gpurun_out/$TAG/pytest_pyr.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest_pyr.log
timeout -k 10 200 python3 -u tools/ab_ops.py pyr 15 base base%HYGRID_PYRSTREAM=0 >> $O 2>&1 || { cat $O; exit 1; }
cat $O
