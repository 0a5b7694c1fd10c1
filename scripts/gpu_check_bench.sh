#!/bin/bash
# GPU test suite, then the bench line twice (no CPU baseline); stops at the first failure
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$i.log 2>&1 || exit $?
  tail -n 1 gpurun_out/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C3", d["value"], d["ms_per_step"], d["kernels_ms"], "roll", d["rollout"]["value"], d["rollout"]["ms_per_step"], "C2", d["c2"]["value"], d["c2"]["ms_per_step"], d["c2"]["kernels_ms"]["step_kernels"], "C2roll", d["c2"]["rollout"]["value"], d["c2"]["rollout"]["ms_per_step"])'
done
