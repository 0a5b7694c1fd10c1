#!/bin/bash
# GPU tests, the default bench line, and step_b in-kernel counters at C5 (prof build). Stops at the
# first failure.
set -u
TAG=${1:-r04d}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/prof_step_b.py > gpurun_out/prof_step_b_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; cat gpurun_out/prof_step_b_${TAG}.log | grep -v amdgpu.ids; exit $rc
