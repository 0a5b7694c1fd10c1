#!/bin/bash
# Run-time knob A/B on the default bench (env line + MAPPO rollout): each entry of AB is
# "NAME:VAR=VAL[,VAR=VAL...]" (NAME only = defaults).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in ${AB:-base}; do
  name=${e%%:*}; vars=""; [ "$e" != "$name" ] && vars=${e#*:}
  env ${vars//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline ${ARGS:-} > gpurun_out/ab_env_$name.log 2>&1 || exit $?
  echo "$name [$vars] $(tail -n 1 gpurun_out/ab_env_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("rollout",{}); print(d["value"], d["ms_per_step"], r.get("value"), r.get("ms_per_step"))')"
done
