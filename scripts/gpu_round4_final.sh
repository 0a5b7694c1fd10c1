#!/bin/bash
# Round 4 final evidence: GPU tests, smoke, the default bench line, then kernel-trace + PMC profiles of
# the C3 and C5 workloads (scripts/gpu_profile.sh). Stops at the first failure.
set -u
TAG=${1:-r04f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
P="--steps 30 --warmup 3 --no-cpu-baseline --rollout-T 0"
TAG=${TAG}c3 WORKLOAD=8x64x5x32768 ARGS="$P --c2-envs 0 --c5-envs 0 --no-ea-line" timeout -k 10 600 bash scripts/gpu_profile.sh > gpurun_out/profile_${TAG}c3.log 2>&1
rc=$?; echo "c3 profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG}c5 WORKLOAD=16x256x5x8192 ARGS="--config c5 $P" timeout -k 10 600 bash scripts/gpu_profile.sh > gpurun_out/profile_${TAG}c5.log 2>&1
rc=$?; echo "c5 profile rc=$rc"; exit $rc
