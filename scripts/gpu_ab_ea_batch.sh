#!/bin/bash
# C2 line (4,096 envs, episode-ahead demand): slots refilled per generation launch (MSC_EA_BATCH) and
# slots per env (MSC_EA_SLOTS)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-b4s12 b2s12 b6s12 b4s16 b8s16 b4s12 b2s12}; do
  b=${v#b}; b=${b%s*}; sl=${v#*s}
  MSC_EA_BATCH=$b MSC_EA_SLOTS=$sl timeout -k 10 300 python bench.py --no-cpu-baseline --rollout-T 0 --steps 50 --warmup 5 > gpurun_out/eab_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/eab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
done
