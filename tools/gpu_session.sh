#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary.
#   tools/gpu_session.sh TAG   -> gpurun_out/TAG/{pytest.log,bench.json,prof/...}
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-images 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
