#!/bin/bash
# C2 two ways on one box: the headline path at --envs 4096, and the bench's c2 line (after a small headline)
set -u
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --envs 4096 --steps 1000 --warmup 1000 --no-cpu-baseline --rollout-T 0 --c2-envs 0 > gpurun_out/c2a_$i.log 2>&1 || exit $?
  echo "headline-path $(tail -n 1 gpurun_out/c2a_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  timeout -k 10 300 python bench.py --envs 1024 --steps 50 --warmup 10 --no-cpu-baseline --rollout-T 0 > gpurun_out/c2b_$i.log 2>&1 || exit $?
  echo "c2-line $(tail -n 1 gpurun_out/c2b_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["c2"]; print(d["value"], d["ms_per_step"])')"
done
