#!/bin/bash
# One GPU call: op A/Bs of variant libraries (tools/ab_ops.py) -> gpurun_out/$1/ab.txt
set -o pipefail
TAG=${1:-ab}; mkdir -p gpurun_out/$TAG; O=gpurun_out/$TAG/ab.txt; : > $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/ab_ops.py conv 15 base cvpd4 cvpd2 cvw5 >> $O 2>&1 || { cat $O; exit 1; }
cat $O
