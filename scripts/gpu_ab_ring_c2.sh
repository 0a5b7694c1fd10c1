#!/bin/bash
# C2 (episode-ahead generation chunks beside the scan allocation): deeper generator rings A/B
set -u
mkdir -p gpurun_out
for v in default ring128q21 ring128q24 default ring128q21 ring128q24; do
  if [ $v = default ]; then var=""; else var=$v; fi
  MSC_LIB_VARIANT=$var timeout -k 10 300 python bench.py --envs 1024 --steps 50 --warmup 10 --no-cpu-baseline --rollout-T 0 > gpurun_out/ringc2_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/ringc2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
done
