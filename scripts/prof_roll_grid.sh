#!/bin/bash
# kernel trace of both rollout lines (C3 MAPPO, C2 IPPO), grouped by (kernel, grid)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rg -o trace --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_rg_bench.log 2>&1 || exit $?
python3 scripts/trace_by_grid.py gpurun_out/prof_rg gpurun_out/kernel_stats_by_grid_rollouts_s2.csv || exit $?
rm -rf gpurun_out/prof_rg
cut -c1-200 gpurun_out/kernel_stats_by_grid_rollouts_s2.csv | head -30
