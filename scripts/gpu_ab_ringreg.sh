#!/bin/bash
# step_c's observation builder with the pending ring read into registers before its stores (8-wave
# blocks, up to 256 VGPRs) vs the ring read between the stores (1024-thread bound, 128 VGPRs)
set -u
mkdir -p gpurun_out
for v in 1 0 1 0; do
  MSC_OBS_RING_REG=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/rr_$v.log 2>&1 || exit $?
  echo "ringreg=$v $(tail -n 1 gpurun_out/rr_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C3", d["value"], d["ms_per_step"], d["kernels_ms"], "roll", d["rollout"]["value"], d["rollout"]["ms_per_step"], "C2", d["c2"]["value"], d["c2"]["ms_per_step"], d["c2"]["kernels_ms"]["step_kernels"], "C2roll", d["c2"]["rollout"]["value"], d["c2"]["rollout"]["ms_per_step"])')"
done
