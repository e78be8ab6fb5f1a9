#!/bin/bash
# End-of-round evidence on one GPU box -> gpurun_out/TAG/: full GPU suite, smoke, the default
# bench line, the rocprofv3 kernel-trace stats of the same bench command (+ per-kernel medians
# of the timed dispatches), and the FETCH_SIZE / WRITE_SIZE traffic passes
# (tools/pmc_traffic.py -> pmc_traffic.json stamped with the kernel-source digest).
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-images 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/bench_kernel_stats.csv" \;
T=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_summary.py "$T" 20 > "$OUT/kernel_medians.json"
timeout -k 10 600 python3 -u tools/pmc_traffic.py "$OUT/pmc" 128 > "$OUT/pmc.log" 2>&1 \
    || { echo "pmc failed"; tail -20 "$OUT/pmc.log"; exit 1; }
cat "$OUT/pmc.log"
