#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roll -o trace --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --rollout-T 100 > gpurun_out/prof_roll_bench.log 2>&1 || exit $?
find gpurun_out/prof_roll -name '*kernel_stats.csv' -exec cp {} gpurun_out/kernel_stats_roll.csv \;
rm -rf gpurun_out/prof_roll
cat gpurun_out/kernel_stats_roll.csv | cut -d, -f1-8 | head -40
