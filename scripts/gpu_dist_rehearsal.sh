#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box: NPROC ranks share the card over gloo (the
# driver's N > 1 runs use RCCL, one rank per GPU); exercises the barriers, the env-id sharding (weak
# and strong: at NPROC = 4 the strong object's ranks own 8,192 of the 32,768 envs each, the regime
# of configs[3] at N = 4: episode-ahead demand + scan allocator), the per-rank episode-ahead memory
# budget of ranks sharing a card, the rollout's advantage-statistics all-reduce and the max-over-ranks
# timing.  usage: [NPROC=4] [ENVS=8192] [STEPS=200] [ROLLOUT_T=100] [OUT=dist_rehearsal_n4] bash scripts/gpu_dist_rehearsal.sh
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
n=${NPROC:-4}
out=${OUT:-dist_rehearsal_n$n}
MSC_DIST_BACKEND=gloo timeout -k 10 ${T_DIST:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $n --envs ${ENVS:-8192} --steps ${STEPS:-200} --warmup 20 \
  --rollout-T ${ROLLOUT_T:-100} --scaling ${SCALING:-both} > gpurun_out/$out.json.log 2>&1
rc=$?; echo "rc=$rc"; tail -n 1 gpurun_out/$out.json.log | cut -c1-600; exit $rc
