#!/bin/bash
# Bench the fused kernel with each variant library: tools/sweep_variants.sh name1 name2 ...
set -o pipefail
mkdir -p gpurun_out/sweep
for v in base "$@"; do
  if [ "$v" = base ]; then unset HYGRID_LIB; else
    export HYGRID_LIB=$PWD/hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd/HyGrid/_lib/variants/libhygrid_$v.so; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-images 0 --no-compare \
      > gpurun_out/sweep/$v.json 2> gpurun_out/sweep/$v.err || { echo "$v failed"; tail -5 gpurun_out/sweep/$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$v.json')); print('$v', d['ms_per_step'], d['kernels'])"
done
