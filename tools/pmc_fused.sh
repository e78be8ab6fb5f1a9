#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over the fused kernel: tools/pmc_fused.sh TAG [stage] [batch]
set -o pipefail
TAG=${1:-pmc}; STAGE=${2:-fused}; B=${3:-32}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
      python3 tools/prof_pipeline.py $STAGE $B 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" k_ > "$OUT/summary.txt"; cat "$OUT/summary.txt"
