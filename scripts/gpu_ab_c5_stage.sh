#!/bin/bash
# C5 (16 x 256 x 5, empirical demand): step_c's observation stage in 3 phases (default) vs unstaged
set -u
mkdir -p gpurun_out
for v in def 0 def 0; do
  if [ $v = def ]; then unset MSC_OBS_STAGE; else export MSC_OBS_STAGE=$v; fi
  timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline --rollout-T 0 --c2-envs 0 > gpurun_out/c5st_$v.log 2>&1 || exit $?
  echo "stage=$v $(tail -n 1 gpurun_out/c5st_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
done
unset MSC_OBS_STAGE
