#!/bin/bash
# Round-3 GPU check of the new / changed kernels -> gpurun_out/TAG/: their tests (verbose),
# in-process A/Bs of the tuning variants, a short bench line with the lattice and wide-conv
# lines.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r03d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_down.py tests/test_gpu_conv_mfma.py \
    tests/test_gpu_pipeline.py tests/test_gpu_fused_conv.py tests/test_gpu_roundtrip.py \
    tests/test_gpu_pyramid.py -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_new.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -2 "$OUT/pytest_new.log"
for ab in "${@:2}"; do
    timeout -k 10 300 python -u tools/ab_ops.py $ab >> "$OUT/ab.txt" 2>&1 || { echo "ab failed: $ab"; tail -5 "$OUT/ab.txt"; exit 1; }
done
[ -f "$OUT/ab.txt" ] && cat "$OUT/ab.txt"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-pyramid --no-roundtrip \
    --no-compare --cpu-images 0 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'],d['roofline']['frac']);print(json.dumps(d['wide_conv']));print(json.dumps(d['lattices']))"
