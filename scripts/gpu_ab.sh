#!/bin/bash
# A/B timing of library variants, one bench line per (variant, repetition); every variant is a set of
# environment assignments (run-time knobs of INTEGRATION.md, or MSC_LIB_VARIANT=<name> for a library
# built with `make variant NAME=<name> VFLAGS=...`). Repetitions alternate the variants (A B A B ...)
# so drift of the box's clock shows up in both.
# usage: VARIANTS="NAME=VAR=val,VAR2=val NAME2=..." [REPS=2] [STEPS=1000] [WARMUP=100] [ROLLOUT_T=0]
#        [BENCH_ARGS="--c2-envs 0 --c5-envs 0 ..."] [RUN_TESTS=0|1] bash scripts/gpu_ab.sh
# Replaces the per-experiment gpu_ab_*.sh drivers of rounds 1-3 (their settings are in DESIGN.md).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${RUN_TESTS:-0}" = 1 ]; then
  timeout -k 10 ${T_TEST:-600} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-default=}; do
    name=${v%%=*}; assigns=${v#*=}
    ( IFS=,; for a in $assigns; do [ -n "$a" ] && export "$a"; done; unset IFS
      timeout -k 10 ${T_BENCH:-300} python bench.py --steps ${STEPS:-1000} --warmup ${WARMUP:-100} --no-cpu-baseline \
        --rollout-T ${ROLLOUT_T:-0} ${BENCH_ARGS:-} > gpurun_out/ab_${name}_$rep.log 2>&1 )
    rc=$?
    echo "== $name rep $rep rc=$rc $(tail -n 1 gpurun_out/ab_${name}_$rep.log | python3 -c 'import json,sys
try:
    d = json.loads(sys.stdin.read())
except Exception:
    print("(no line)"); sys.exit(0)
o = [d["value"], d["ms_per_step"], d["kernels_ms"]]
for k in ("rollout", "c2", "c5"):
    if k in d:
        o += [k, d[k]["value"], d[k]["ms_per_step"]]
print(*o)')"
    [ $rc -eq 0 ] || exit $rc
  done
done
