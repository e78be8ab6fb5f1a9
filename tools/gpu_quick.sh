#!/bin/bash
# Quick GPU check: pipeline parity tests, then a short fused bench.
#   tools/gpu_quick.sh [pytest-target]
set -o pipefail
T=${1:-tests/test_gpu_pipeline.py}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-images 0 --no-compare --steps 20 2> gpurun_out/quick_bench.err
