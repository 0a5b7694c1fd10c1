#!/bin/bash
# C3 env line + MAPPO rollout line with step_c's observation staging on (default) / off
set -u
mkdir -p gpurun_out
for st in 1 0 1 0; do
  MSC_OBS_STAGE=$st timeout -k 10 300 python bench.py --no-cpu-baseline --c2-envs 0 > gpurun_out/stage_$st.log 2>&1 || exit $?
  echo "stage=$st $(tail -n 1 gpurun_out/stage_$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"], d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
