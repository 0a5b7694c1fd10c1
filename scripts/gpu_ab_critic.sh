#!/bin/bash
# rollout lines (C3 MAPPO, C2 IPPO): critic on the main stream / on a side stream issued before the
# actor / on a side stream issued after the sampling kernel (beside the env step)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-main side late main side late}; do
  case $v in
    main) envs="MSC_ROLLOUT_CRITIC_SIDE=0";; side) envs="MSC_ROLLOUT_CRITIC_SIDE=1";;
    late) envs="MSC_ROLLOUT_CRITIC_SIDE=1 MSC_ROLLOUT_CRITIC_LATE=1";;
  esac
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/cr_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/cr_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C3 rollout", d["rollout"]["value"], d["rollout"]["ms_per_step"], "C2 rollout", d["c2"]["rollout"]["value"], d["c2"]["rollout"]["ms_per_step"])')"
done
