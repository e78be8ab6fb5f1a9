#!/bin/bash
# Fused-kernel investigation on one GPU box -> gpurun_out/TAG/
#   1. issue-rate microbenchmark (tools/microbench/issue, built on the CPU host)
#   2. interleaved in-process A/B of fused-kernel variants (tools/ab_fused.py)
#   3. SQ PMC passes over the in-tree fused kernel (tools/pmc_fused.sh)
# usage: tools/probe_fused.sh TAG "variant names for ab_fused" [extra SQ counters pass]
set -o pipefail
TAG=${1:-probe}; VARS=${2:-base}; P3=${3:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -x tools/microbench/issue ]; then
  timeout -k 10 120 tools/microbench/issue > "$OUT/issue.txt" 2>&1 || { echo "issue failed"; tail -5 "$OUT/issue.txt"; exit 1; }
  echo "issue ok"
fi
timeout -k 10 300 python3 -u tools/ab_fused.py 15 $VARS > "$OUT/ab.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter list failed (continuing)"
bash tools/pmc_fused.sh "$TAG/pmc" fused 32 || exit 1
if [ -n "$P3" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $P3 --output-format csv -d "$OUT/pmc/p3" -o run -- \
      python3 tools/prof_pipeline.py fused 32 2 > "$OUT/pmc/p3.log" 2>&1 || { echo "pass 3 failed"; tail -5 "$OUT/pmc/p3.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc" k_ > "$OUT/pmc/summary.txt"; cat "$OUT/pmc/summary.txt"
fi
