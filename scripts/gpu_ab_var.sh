#!/bin/bash
# Library-variant A/B (make variant NAME=...): bench lines for the default build and each variant.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${VARIANTS:-default}; do
  for a in ${CONFIGS:-c5}; do
    if [ "$a" = c5 ]; then args="--config c5"; elif [ "$a" = c2 ]; then args="--envs 4096"; else args=""; fi
    vv=$v; [ "$v" = default ] && vv=""
    MSC_LIB_VARIANT=$vv timeout -k 10 300 python bench.py $args --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --rollout-T 0 > gpurun_out/ab_${v}_$a.log 2>&1 || exit $?
    echo "$v $a $(tail -n 1 gpurun_out/ab_${v}_$a.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
  done
done
