#!/bin/bash
# Train + evaluate with the reference's scripts/run_experiment.sh arguments on MI355X.
# The reference's script starts Ray under SLURM and calls src/experiments/run_experiment.py; here
# the same two calls (--mode single, then --mode evaluate) go to marlsc.experiment, which runs the
# envs, the rollout and the PPO learner on the GPU (torchrun: one process per GPU when NGPUS > 1).
#
# Override with environment variables:
#   ENV_CONFIG ALGO_CONFIG STORAGE_DIR EXPERIMENT_NAME ROOT_SEED EVAL_EPISODES NGPUS EXTRA_ARGS
# The algorithm YAMLs carry the reference's sampling setup (2 runners x 10 envs); on the GPU pass
# the env count per GPU, e.g. EXTRA_ARGS="--envs 4096" (BASELINE configs[1]).
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH="$(pwd)/marl-sc_amd${PYTHONPATH:+:$PYTHONPATH}"
export PYTHONUNBUFFERED=1
export PYTHONHASHSEED=0

ENV_CONFIG=${ENV_CONFIG:-./config_files/environments/env_c3_8wh64r5sku.yaml}
ALGO_CONFIG=${ALGO_CONFIG:-./config_files/algorithms/mappo.yaml}
STORAGE_DIR=${STORAGE_DIR:-./experiment_outputs}
EXPERIMENT_NAME=${EXPERIMENT_NAME:-MAPPO_8WH64R5SKU}
ROOT_SEED=${ROOT_SEED:-42}
EVAL_EPISODES=${EVAL_EPISODES:-100}
NGPUS=${NGPUS:-1}
EXTRA_ARGS=${EXTRA_ARGS:-}

if [ "$NGPUS" -gt 1 ]; then
  LAUNCH=(python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPUS" --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29517}" -m)
else
  LAUNCH=(python -m)
fi

# Run training
"${LAUNCH[@]}" marlsc.experiment \
    --mode single \
    --env-config "${ENV_CONFIG}" \
    --algorithm-config "${ALGO_CONFIG}" \
    --storage-dir "${STORAGE_DIR}" \
    --experiment-name "${EXPERIMENT_NAME}" \
    --root-seed "${ROOT_SEED}" ${EXTRA_ARGS}

# Run evaluation
python -m marlsc.experiment \
    --mode evaluate \
    --storage-dir "${STORAGE_DIR}" \
    --experiment-name "${EXPERIMENT_NAME}" \
    --eval-episodes "${EVAL_EPISODES}" \
    --root-seed "${ROOT_SEED}"
