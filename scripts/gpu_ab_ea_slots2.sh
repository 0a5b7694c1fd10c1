#!/bin/bash
# C2 line (24 episodes after 24) and its IPPO rollout: 16 / 20 / 24 / 32 episode-ahead slots, 4 per refill
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-16 24 32 20 16 24}; do
  MSC_EA_SLOTS=$v MSC_EA_BATCH=4 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/eas2_$v.log 2>&1 || exit $?
  echo "slots=$v $(tail -n 1 gpurun_out/eas2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"], d["kernels_ms"], "roll", d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
