#!/bin/bash
# Round 4 evidence, part 1: GPU tests, smoke, the default bench line. Stops at the first failure.
set -u
TAG=${1:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
