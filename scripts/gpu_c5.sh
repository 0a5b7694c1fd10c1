#!/bin/bash
# GPU tests and the C5 line alone (A/B of step_b changes). Stops at the first failure.
set -u
TAG=${1:-c5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
timeout -k 10 300 python bench.py --config c5 --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_${TAG}_$rep.json.log 2>&1
rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/bench_${TAG}_$rep.json.log') if l.startswith('{')][0];print('C5', round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms'])"
done
exit 0
