#!/bin/bash
# One GPU-box session: parity tests, smoke, bench. Stops at the first GPU fault / timeout.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures (no fault)
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 3 gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/bench.log
exit $rc
