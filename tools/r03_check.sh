#!/bin/bash
# Round-3 GPU check: the new / changed tests first (verbose), then the whole GPU suite, smoke
# and a bench line.  -> gpurun_out/TAG/
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_pipeline.py \
    tests/test_gpu_roundtrip.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_new.log" 2>&1 || { echo "new tests failed"; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -2 "$OUT/pytest_new.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
