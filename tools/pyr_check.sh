set -o pipefail
mkdir -p gpurun_out/pyr
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pyr/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/pyr/pytest.log
for op in pyrfr pyr pyr1; do timeout -k 10 200 python tools/ab_ops.py $op 20 base base%HYGRID_PYR_KERNEL=stream >> gpurun_out/pyr/ab.txt 2>&1 || exit 1; done
cat gpurun_out/pyr/ab.txt
exit $rc
