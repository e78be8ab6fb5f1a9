#!/bin/bash
# A microbenchmark binary timed, then its kernel trace and FETCH_SIZE / WRITE_SIZE passes
# (one rocprofv3 run per pass, the binary directly after `--`), counters per kernel:
#   tools/mb_pmc.sh TAG NAME ALG_BYTES [ARGS for the timed run] -- [ARGS for the profiled runs]
# -> gpurun_out/TAG/{time.txt,stats,fetch,write,pmc.txt}
set -o pipefail
TAG=$1; NAME=$2; ALG=$3; shift 3
TARGS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do TARGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
PARGS=("$@")
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
B=tools/microbench/$NAME
timeout -k 10 240 "$B" "${TARGS[@]}" > "$OUT/time.txt" 2>&1 || { echo "timed run failed"; tail -5 "$OUT/time.txt"; exit 1; }
cat "$OUT/time.txt"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- "$B" "${PARGS[@]}" \
    > "$OUT/stats.log" 2>&1 || { echo "stats pass failed"; tail -5 "$OUT/stats.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "$B" "${PARGS[@]}" \
    > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -5 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "$B" "${PARGS[@]}" \
    > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -5 "$OUT/write.log"; exit 1; }
{
  echo "== FETCH_SIZE x2 (gfx950 correction) vs $ALG B / 2 (reads)"
  python3 tools/pmc_by_kernel.py "$OUT/fetch" FETCH_SIZE "$(python3 -c "print($ALG/2)")" x2
  echo "== FETCH_SIZE raw vs reads"
  python3 tools/pmc_by_kernel.py "$OUT/fetch" FETCH_SIZE "$(python3 -c "print($ALG/2)")"
  echo "== WRITE_SIZE vs $ALG B / 2 (writes)"
  python3 tools/pmc_by_kernel.py "$OUT/write" WRITE_SIZE "$(python3 -c "print($ALG/2)")"
} > "$OUT/pmc.txt"
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cat "$OUT/pmc.txt"
