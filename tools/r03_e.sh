#!/bin/bash
# Round-3: pyramid-level tests + A/B of the LDS vertex gather (gpurun_out/TAG/)
set -o pipefail
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_roundtrip.py -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for op in pyrfr pyr pyr1; do
    timeout -k 10 300 python -u tools/ab_ops.py $op 30 base pd0 >> "$OUT/ab.txt" 2>&1 \
        || { echo "ab failed"; tail -5 "$OUT/ab.txt"; exit 1; }
done
cat "$OUT/ab.txt"
