#!/bin/bash
# One GPU call: pyramid parity tests + the pyramid path A/B (tools/ab_pyramid.py) -> gpurun_out/$1/
set -o pipefail
TAG=${1:-ab}; mkdir -p gpurun_out/$TAG; O=gpurun_out/$TAG/ab.txt; : > $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pyramid.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python3 -u tools/ab_pyramid.py 10 8 >> $O 2>&1 || { cat $O; exit 1; }
cat $O
