#!/bin/bash
# the default bench line twice on one box: headline, rollout, c2 and c2 rollout values
set -u
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/full_$i.log 2>&1 || exit $?
  echo "full $i $(tail -n 1 gpurun_out/full_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["rollout"]["value"], d["c2"]["value"], d["c2"]["ms_per_step"], d["c2"]["rollout"]["value"])')"
done
