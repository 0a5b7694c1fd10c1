#!/bin/bash
# C3 demand kernel: deeper generator rings (128 positions, fewer demand blocks per CU) with a quota
# near the mean consumption against the default 64-position ring, quota 24
set -u
mkdir -p gpurun_out
for v in default ring128q21 ring128q18 ring128q24 default ring128q21; do
  if [ $v = default ]; then var=""; else var=$v; fi
  MSC_LIB_VARIANT=$var timeout -k 10 300 python bench.py --no-cpu-baseline --rollout-T 0 --c2-envs 0 > gpurun_out/ring_$v.log 2>&1 || exit $?
  echo "$v $(tail -n 1 gpurun_out/ring_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
done
