#!/bin/bash
# Round-2 evidence: GPU parity tests, rocprofv3 kernel stats + PMC passes (scripts/gpu_profile.sh),
# the ISA issue-cost microbenchmark, then the default bench line. Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/ubench_isa > gpurun_out/ubench_isa.txt 2>&1 || exit $?
TAG=${TAG:-r02} bash scripts/gpu_profile.sh > gpurun_out/profile.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/bench.log; exit $rc
