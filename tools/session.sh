#!/bin/bash
# One GPU-box session, parametrised (replaces the per-round one-off scripts):
#   tools/session.sh TAG STEP [STEP ...]        -> gpurun_out/TAG/
# Each STEP is one quoted word list, run in order; the first failure ends the session
# (no GPU step runs after a failed, aborted or timed-out one):
#   "test FILE..."          pytest on those files (verbose tail, per-test timeout)
#   "gputests"              the whole -m gpu suite
#   "smoke"                 __graft_entry__.smoke()
#   "bench [ARGS...]"       bench.py (default: the driver's --steps 20 --warmup 5)
#   "ab TOOL ARGS..."       tools/TOOL.py ARGS (in-process A/B of library variants)
#   "py SCRIPT ARGS..."     any tools/ python script (prof drivers, microbench drivers)
#   "sq STAGE BATCH"        SQ counter passes of tools/prof_pipeline.py STAGE (tools/pmc_fused.sh)
#   "pmc KERNEL CMD..."     FETCH/WRITE + SQ passes over one kernel (tools/pmc_kernel.sh)
#   "final"                 end-of-round evidence (tools/final_session.sh) + fused SQ passes
#   "mb NAME ARGS..."       run a microbenchmark binary tools/microbench/NAME (built on the host)
#   "mbpmc NAME ALG ARGS"   the same, then its kernel trace + FETCH/WRITE passes (tools/mb_pmc.sh)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for S in "$@"; do
    n=$((n + 1))
    set -- $S
    kind=$1; shift
    log="$OUT/$(printf %02d $n)_$kind${1:+_$(basename "$1" .py)}.txt"
    echo "== [$n] $S" | tee "$log"
    case $kind in
    test)  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" \
               >> "$log" 2>&1; rc=$?; tail -4 "$log" ;;
    gputests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
               >> "$log" 2>&1; rc=$?; tail -3 "$log" ;;
    smoke) timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" >> "$log" 2>&1; rc=$?
           tail -2 "$log" ;;
    bench) [ $# -eq 0 ] && set -- --steps 20 --warmup 5
           timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench_$n.json" 2>> "$log"; rc=$?
           cat "$OUT/bench_$n.json" | tee -a "$log" ;;
    ab)    tool=$1; shift
           timeout -k 10 400 python -u tools/$tool.py "$@" 2>&1 | grep -v amdgpu.ids >> "$log"; rc=$?
           cat "$log" ;;
    py)    tool=$1; shift
           timeout -k 10 400 python -u tools/$tool "$@" >> "$log" 2>&1; rc=$?; tail -40 "$log" ;;
    sq)    bash tools/pmc_fused.sh "$TAG/sq_$n" "$@" >> "$log" 2>&1; rc=$?; tail -30 "$log" ;;
    pmc)   k=$1; shift
           bash tools/pmc_kernel.sh "$TAG/pmc_$n" "$k" -- "$@" >> "$log" 2>&1; rc=$?
           grep -E "FETCH|WRITE|WAIT|WAVE_CYCLES|VMEM|VALU|ACTIVE_INST_ANY|BANK" "$log" ;;
    final) bash tools/final_session.sh "$TAG/final" >> "$log" 2>&1 && \
               bash tools/pmc_fused.sh "$TAG/final/sq" fused 32 >> "$log" 2>&1; rc=$?; tail -30 "$log" ;;
    mb)    b=$1; shift
           timeout -k 10 300 tools/microbench/$b "$@" >> "$log" 2>&1; rc=$?; tail -30 "$log" ;;
    mbpmc) bash tools/mb_pmc.sh "$TAG/mbpmc_$n" "$@" >> "$log" 2>&1; rc=$?; tail -40 "$log" ;;
    *)     echo "unknown step kind: $kind"; rc=2 ;;
    esac
    if [ $rc -ne 0 ]; then echo "step $n failed (rc $rc): $S"; exit $rc; fi
done
echo "session $TAG: $n steps ok"
