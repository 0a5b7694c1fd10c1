#!/bin/bash
# C3 MAPPO rollout (chain-bound: step_a -> allocation -> step_c -> actor) with each allocation kernel:
# lane (default at 32768 envs), lane with 2 / 4 lanes per env, group (8 lanes per env), scan (a wave per env)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-lane lpe2 lpe4 group scan lane}; do
  case $v in
    lane) envs="MSC_ALLOC_IMPL=lane";; lpe2) envs="MSC_ALLOC_IMPL=lane MSC_ALLOC_LPE=2";;
    lpe4) envs="MSC_ALLOC_IMPL=lane MSC_ALLOC_LPE=4";; group) envs="MSC_ALLOC_IMPL=group";; scan) envs="MSC_ALLOC_IMPL=scan";;
  esac
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --c2-envs 0 --steps 300 --warmup 50 > gpurun_out/ra_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/ra_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"], d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
