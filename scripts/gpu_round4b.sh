#!/bin/bash
# Round 4 evidence, part 2: profiles (kernel trace + PMC passes) of each workload with nothing else of
# the same grid in the run: C3 per-step (no episode-ahead line), C3 episode-ahead steady state (only
# its generation kernel kept), C2 (the headline shrunk to 32 envs, below the C2 grids), C5.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
P="--steps 30 --warmup 3 --no-cpu-baseline --rollout-T 0"
TAG=r04c3 WORKLOAD=8x64x5x32768 ARGS="$P --c2-envs 0 --c5-envs 0 --no-ea-line" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/profile_r04c3.log 2>&1 || exit $?
echo "c3 ok"
TAG=r04c3ea WORKLOAD=8x64x5x32768 PMC_ONLY=demand_unit_kernel_ea ARGS="$P --c2-envs 0 --c5-envs 0" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/profile_r04c3ea.log 2>&1 || exit $?
echo "c3ea ok"
TAG=r04c2 WORKLOAD=8x64x5x4096 ARGS="$P --c5-envs 0 --no-ea-line --envs 32" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/profile_r04c2.log 2>&1 || exit $?
echo "c2 ok"
TAG=r04c5 WORKLOAD=16x256x5x8192 ARGS="--config c5 $P" timeout -k 10 900 bash scripts/gpu_profile.sh > gpurun_out/profile_r04c5.log 2>&1 || exit $?
echo "c5 ok"
