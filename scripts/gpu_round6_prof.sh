#!/bin/bash
# Round 6 evidence from the committed build: GPU tests, then the round's profile set (C3, C2, C5:
# scripts/gpu_profile_all.sh) and the C3 episode-ahead steady-state profile (the EA line's refill
# launches, PMC_ONLY=demand_v3_kernel_ea). Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r06p.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_r06p.log; [ $rc -eq 0 ] || exit $rc
fi
R=${R:-r06} timeout -k 10 2400 bash scripts/gpu_profile_all.sh || exit $?
TAG=${R:-r06}c3ea PMC_ONLY=demand_v3_kernel_ea ARGS="--steps 30 --warmup 3 --no-cpu-baseline --rollout-T 0 --c2-envs 0 --c5-envs 0 --scaling weak" \
  timeout -k 10 1200 bash scripts/gpu_profile.sh > /dev/null || exit $?
echo "c3ea done"
