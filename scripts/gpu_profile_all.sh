#!/bin/bash
# The round's profile set: scripts/gpu_profile.sh for C3 (per-step pipelined demand), C2 (4,096 envs)
# and C5 (16 x 256 x 5, empirical trace), tags ${R}c3 / ${R}c2 / ${R}c5. Stops at the first failure.
set -u
R=${R:-r05}
COMMON="--no-cpu-baseline --rollout-T 0 --c2-envs 0 --c5-envs 0 --no-ea-line"
TAG=${R}c3 ARGS="--steps 30 --warmup 3 $COMMON" bash scripts/gpu_profile.sh > /dev/null || exit $?
echo "c3 done"
TAG=${R}c2 WORKLOAD=8x64x5x4096 ARGS="--steps 300 --warmup 600 --envs 4096 $COMMON" \
  bash scripts/gpu_profile.sh > /dev/null || exit $?
echo "c2 done"
TAG=${R}c5 WORKLOAD=16x256x5x8192 ARGS="--config c5 --steps 100 --warmup 10 $COMMON" \
  bash scripts/gpu_profile.sh > /dev/null || exit $?
echo "c5 done"
