#!/bin/bash
# step_c observation staging in P phases (MSC_OBS_STAGE = P): parity tests with P = 2 and 3, then the
# C3 env + MAPPO rollout lines for P = 1 / 2 / 4
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 2 3; do
  MSC_OBS_STAGE=$P timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_stage$P.log 2>&1
  rc=$?; echo "parity P=$P rc=$rc $(tail -n 1 gpurun_out/pt_stage$P.log)"; [ $rc -eq 0 ] || exit $rc
done
for P in 1 2 4 1 2 4; do
  MSC_OBS_STAGE=$P timeout -k 10 400 python bench.py --no-cpu-baseline --c2-envs 0 > gpurun_out/stp_$P.log 2>&1 || exit $?
  echo "stage=$P $(tail -n 1 gpurun_out/stp_$P.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"], "roll", d["rollout"]["value"], d["rollout"]["ms_per_step"])')"
done
