#!/bin/bash
# C5 scan allocator (16 warehouses, two SKU slots per lane): GPU tests, default bench line, and the
# C5 line with the group allocator forced (A/B). Stops at the first failure.
set -u
TAG=${1:-c5scan}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
MSC_ALLOC_IMPL=group timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/bench_${TAG}_c5group.json.log 2>&1
rc=$?; echo "c5 group rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/bench_${TAG}_c5scan.json.log 2>&1
rc=$?; echo "c5 scan rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/host_overhead.py > gpurun_out/host_${TAG}.log 2>&1
rc=$?; echo "host rc=$rc"; cat gpurun_out/host_${TAG}.log | grep us/step; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --hip-runtime-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hostprof_${TAG} -o host -- python $GRAFT_REPO_ROOT/tools/host_overhead.py 20 25 > $GRAFT_REPO_ROOT/gpurun_out/hostprof_${TAG}.log 2>&1
rc=$?; echo "hostprof rc=$rc"; exit $rc
