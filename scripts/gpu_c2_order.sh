#!/bin/bash
# c2 line after the full bench's earlier phases: EA stream queue priority A/B
set -u
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 600 env "$@" > gpurun_out/o_$tag.log 2>&1 || exit $?
  echo "$tag $(tail -n 1 gpurun_out/o_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["c2"]["value"], d["c2"]["ms_per_step"], d["c2"]["host_ms_per_step"])')"; }
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
run default python bench.py --no-cpu-baseline --steps 50 --warmup 10
run low MSC_EA_PRIO=low python bench.py --no-cpu-baseline --steps 50 --warmup 10
run high MSC_EA_PRIO=high python bench.py --no-cpu-baseline --steps 50 --warmup 10
run lownorollout MSC_EA_PRIO=low python bench.py --no-cpu-baseline --steps 50 --warmup 10 --rollout-T 0
