#!/bin/bash
# One GPU-box session of a build step: a subset of the GPU tests (PYTEST_K), A/B bench lines
# (scripts/gpu_ab.sh: VARIANTS, REPS, STEPS, BENCH_ARGS), optionally the two-rank gloo rehearsal (DIST=1)
# and a bench line (BENCH=1, FINAL_ARGS). Every GPU
# step runs under its own time limit; the session stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-s}
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 ${T_TEST:-600} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q -p no:cacheprovider --timeout 200 \
    --timeout-method thread -k "$PYTEST_K" > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/${tag}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${VARIANTS:-}" ]; then
  bash scripts/gpu_ab.sh || exit $?
fi
if [ "${DIST:-0}" = 1 ]; then
  MSC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --envs ${DIST_ENVS:-8192} --steps 200 --warmup 20 \
    --rollout-T 20 > gpurun_out/${tag}_dist.log 2>&1
  rc=$?; echo "dist rc=$rc"; tail -n 1 gpurun_out/${tag}_dist.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 ${T_BENCH:-600} python bench.py ${FINAL_ARGS:-} > gpurun_out/${tag}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/${tag}_bench.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
