#!/bin/bash
# A/B timing of library variants selected by environment variables (one bench line each).
# usage: VARIANTS="NAME=VAR=val,VAR2=val NAME2=..." [T_TEST=..] [RUN_TESTS=1] bash scripts/gpu_ab.sh
set -u
mkdir -p gpurun_out
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 ${T_TEST:-600} python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for v in ${VARIANTS:-default=}; do
  name=${v%%=*}; assigns=${v#*=}
  ( IFS=,; for a in $assigns; do [ -n "$a" ] && export "$a"; done; unset IFS
    timeout -k 10 ${T_BENCH:-300} python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --rollout-T ${ROLLOUT_T:-100} ${BENCH_ARGS:-} > gpurun_out/ab_$name.log 2>&1 )
  rc=$?; echo "== $name rc=$rc"; grep -o '"ms_per_step[^,]*\|"kernels_ms": {[^}]*}' gpurun_out/ab_$name.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
