#!/bin/bash
# Round-2 evidence run on one GPU box: full GPU suite, smoke, the default bench line and the
# rocprofv3 kernel-trace summary of the same bench command.   -> gpurun_out/TAG/
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --cpu-images 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/bench_kernel_stats.csv" \;
cut -d, -f1-5 "$OUT/bench_kernel_stats.csv" | cut -c1-160
