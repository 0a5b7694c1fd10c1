#!/bin/bash
# Fused MLP output-layer A/B (VALU vs MFMA) x layer-2 tiles per pass: rollout tests, then
# bench lines (rollout + the MLP alone).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_train.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_mlp2.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${AB_CFGS:-1:8 0:8 1:2 0:2 1:8 1:2}; do
  set -- ${cfg%:*} ${cfg#*:}
  MSC_MLP_V3=$1 MSC_MLP_P8=$2 timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/ab_mlp2_$1_$2.log 2>&1 || exit $?
  echo "v3=$1 p8=$2 $(tail -n 1 gpurun_out/ab_mlp2_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline_mlp"]; print(d["rollout"]["value"], d["rollout"]["ms_per_step"], r["ms"], r["achieved"], r["frac"])')"
done
