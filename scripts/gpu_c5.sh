#!/bin/bash
# C5 / allocation-order A/B: GPU parity tests, then bench --config c5 with and without the
# order-count sort of the group allocation kernel, and the C2 shape (Poisson, 4096 envs).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${AB_CFGS:-c5:1 c5:0 c2:1 c2:0 c5:1}; do
  set -- ${cfg%:*} ${cfg#*:}
  if [ "$1" = c5 ]; then args="--config c5"; else args="--envs 4096"; fi
  MSC_ALLOC_SORT=$2 timeout -k 10 300 python bench.py $args --steps 200 --warmup 20 --no-cpu-baseline --rollout-T 0 > gpurun_out/ab_sort_$1_$2.log 2>&1 || exit $?
  echo "$1 sort=$2 $(tail -n 1 gpurun_out/ab_sort_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
done
