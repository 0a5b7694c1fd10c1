#!/bin/bash
# A/B of the episode-ahead chunk length (MSC_EA_CHUNK steps per generation launch) on the C2 line
set -u
mkdir -p gpurun_out
for ch in ${CHUNKS:-10 5 20 10 5 20}; do
  MSC_EA_CHUNK=$ch timeout -k 10 300 python bench.py --envs 4096 --steps 1000 --warmup 1000 --no-cpu-baseline --rollout-T 0 --c2-envs 0 > gpurun_out/ab_ch_$ch.log 2>&1 || exit $?
  echo "chunk $ch $(tail -n 1 gpurun_out/ab_ch_$ch.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
