#!/bin/bash
# Fused policy MLP (csrc/mlp.hip): GPU tests, rollout A/B and a rocprofv3 kernel-stats pass.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_mlp.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${AB_CFGS:-8:1 4:1 8:1}; do
  set -- ${cfg%:*} ${cfg#*:}
  MSC_MLP_P8=$1 MSC_MLP_PRIO=$2 timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/ab_mlp_$1_$2.log 2>&1 || exit $?
  echo "p8=$1 prio=$2 $(tail -n 1 gpurun_out/ab_mlp_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline_mlp"]; print(d["rollout"]["value"], d["rollout"]["ms_per_step"], r["ms"], r["achieved"], r["frac"])')"
done
[ "${PROF:-1}" = "1" ] || exit 0
bash scripts/prof_roll.sh > gpurun_out/prof_roll.txt 2>&1 || exit $?
