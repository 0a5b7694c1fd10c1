#!/bin/bash
# C2 with episode-ahead demand: step_a / step_c wave priority A/B over whole refill periods
set -u
mkdir -p gpurun_out
for v in 1 0 1 0; do
  MSC_CHAIN_PRIO=$v timeout -k 10 300 python bench.py --envs 1024 --steps 50 --warmup 10 --no-cpu-baseline --rollout-T 0 > gpurun_out/cp_$v.log 2>&1 || exit $?
  echo "chain_prio $v $(tail -n 1 gpurun_out/cp_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"], d["steps"], d["kernels_ms"])')"
done
