#!/bin/bash
# Rollout A/B: env lanes on separate HIP streams (bench.py --rollout-lanes) and library pipelining.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${AB_CFGS:-1:1 2:1 2:0 4:1 1:1 2:1}; do
  set -- ${cfg%:*} ${cfg#*:}
  MSC_ROLLOUT_PIPELINE=$2 timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --rollout-lanes $1 > gpurun_out/ab_roll_$1_$2.log 2>&1 || exit $?
  echo "lanes=$1 pipe=$2 $(tail -n 1 gpurun_out/ab_roll_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
