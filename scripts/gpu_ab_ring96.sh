#!/bin/bash
# C3 env step: a 96-position generator ring (two 53-KB demand blocks per CU) with the allocation
# block shrunk to fit beside them (cost table read from L2, 6-order record windows: 27 KB) against
# the default 64-position ring; pipelined and sequential (MSC_PIPELINE=0: each kernel alone)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-default notab6 r96q21 r96q24 default r96q21}; do
  if [ $v = default ]; then var=""; else var=$v; fi
  for pl in 1 0; do
    MSC_PIPELINE=$pl MSC_LIB_VARIANT=$var timeout -k 10 300 python bench.py --no-cpu-baseline --rollout-T 0 --c2-envs 0 --steps ${STEPS:-1000} > gpurun_out/ab96_${v}_$pl.log 2>&1 || exit $?
    echo "$v pipeline=$pl $(tail -n 1 gpurun_out/ab96_${v}_$pl.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
  done
done
