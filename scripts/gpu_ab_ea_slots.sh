#!/bin/bash
# C2 line over 48 episodes (4,800 steps) after 12: episode-ahead slots per env 12 / 16 (4 per launch),
# env line and IPPO rollout
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-12 16 12 16}; do
  MSC_EA_SLOTS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4800 --warmup 5 > gpurun_out/eas_$v.log 2>&1 || exit $?
  echo "slots=$v $(tail -n 1 gpurun_out/eas_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"], d["steps"], d["kernels_ms"], "roll", d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
