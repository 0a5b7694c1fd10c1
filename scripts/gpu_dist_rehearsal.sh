#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box: 2 ranks share the card over gloo (the
# driver's N > 1 runs use RCCL, one rank per GPU); exercises the barriers, the env-id sharding,
# the rollout's advantage-statistics all-reduce and the max-over-ranks timing.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
MSC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --envs 8192 --steps 50 --warmup 10 --rollout-T 20 > gpurun_out/dist_rehearsal.log 2>&1
rc=$?; echo "rc=$rc"; tail -n 1 gpurun_out/dist_rehearsal.log | cut -c1-600; exit $rc
