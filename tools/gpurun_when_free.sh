#!/bin/bash
# Submit one gpurun call, waiting for a free GPU slot: resubmits ONLY while gpurun reports
# "no box or slot free" (exit 3: nothing ran, nothing charged), at most N times, 4 min apart.
# Any other outcome (success, failure, refusal) ends it.  Never used to retry a GPU step.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command' [N]
LOG=$1; TO=$2; CMD=$3; N=${4:-8}
for i in $(seq 1 "$N"); do
    timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy" "$LOG"; then
        echo "gpurun rc=$rc (attempt $i)" >> "$LOG"
        exit $rc
    fi
    sleep 240
done
echo "no GPU slot after $N attempts" >> "$LOG"
exit 3
