"""CLI of the reference's experiment entry point (src/experiments/run_experiment.py), for the modes
that drive this build's training path: `single` (train one seed, with periodic evaluation and
checkpoints) and `evaluate` (deterministic episodes from a checkpoint). Ray Tune sweeps, seed
evaluation and W&B are out of scope; their flags are accepted and ignored.

    python -m marlsc.experiment --mode single --env-config ENV.yaml --algorithm-config ALGO.yaml \
        --storage-dir ./experiment_outputs --experiment-name NAME --root-seed 42
    python -m marlsc.experiment --mode evaluate --storage-dir ./experiment_outputs \
        --experiment-name NAME --eval-episodes 100 --root-seed 42

Multi-GPU: launch `single` with torchrun (one process per GPU, RCCL); each rank owns
`--envs` envs (global env ids), gradients and advantage statistics are all-reduced.
Output layout (per experiment): config_env.yaml, config_algorithm.yaml, run_metadata.json,
training_metrics.jsonl, checkpoints/checkpoint_NNNNNN/, checkpoints/checkpoint_final/,
eval_results.json (evaluate mode).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time
from pathlib import Path
from typing import Any, Dict, List, Optional

import yaml

DEFAULT_EVAL_EPISODES = 10


def parse_args(argv: Optional[List[str]] = None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--mode", choices=["single", "evaluate"], default="single")
    ap.add_argument("--env-config")
    ap.add_argument("--algorithm-config")
    ap.add_argument("--storage-dir", default="./experiment_outputs")
    ap.add_argument("--experiment-name")
    ap.add_argument("--root-seed", type=int, default=None)
    ap.add_argument("--eval-seed", type=int, default=None)
    ap.add_argument("--eval-episodes", type=int, default=None)
    ap.add_argument("--resume-from", default=None, help="checkpoint directory to continue training from")
    ap.add_argument("--checkpoint", default=None, help="evaluate: checkpoint directory (default: the final one)")
    ap.add_argument("--num-iterations", type=int, default=None, help="override shared.num_iterations")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: num_envs_per_env_runner)")
    ap.add_argument("--rollout-len", type=int, default=None, help="env steps per rollout (default: from batch_size)")
    ap.add_argument("--device", type=int, default=None)
    # accepted for command-line compatibility with the reference, no effect here
    ap.add_argument("--wandb-project", default=None)
    ap.add_argument("--wandb-name", default=None)
    ap.add_argument("--visualize", action="store_true")
    return ap.parse_args(argv)


def _dist_setup():
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return (dist.get_rank() if world > 1 else 0), world, local


def _load_configs(env_path: str, algo_path: str):
    from .config import load_environment_config
    from .ppo import PPOConfig
    env_cfg = load_environment_config(env_path, allow_nr_ne_nw=True)
    algo_raw = yaml.safe_load(open(algo_path))
    return env_cfg, algo_raw, PPOConfig.from_algorithm_config(algo_raw)


def run_single(args) -> Dict[str, Any]:
    from .ppo import PPOTrainer
    rank, world, local = _dist_setup()
    device = local if args.device is None else args.device
    if not args.env_config or not args.algorithm_config:
        raise SystemExit("--env-config and --algorithm-config are required for --mode single")
    env_cfg, algo_raw, cfg = _load_configs(args.env_config, args.algorithm_config)
    if args.num_iterations is not None:
        cfg.num_iterations = args.num_iterations
    root_seed = 42 if args.root_seed is None else args.root_seed
    name = args.experiment_name or f"{cfg.name.upper()}_{Path(args.env_config).stem}_seed{root_seed}"
    out = Path(args.storage_dir) / name
    trainer = PPOTrainer(env_cfg, cfg, root_seed=root_seed, n_envs=args.envs, rollout_len=args.rollout_len,
                         device=device, eval_seed=args.eval_seed)
    if args.resume_from:
        trainer.load_checkpoint(args.resume_from)
    if rank == 0:
        (out / "checkpoints").mkdir(parents=True, exist_ok=True)
        shutil.copyfile(args.env_config, out / "config_env.yaml")
        shutil.copyfile(args.algorithm_config, out / "config_algorithm.yaml")
        (out / "run_metadata.json").write_text(json.dumps({
            "root_seed": root_seed, "train_seed": trainer.train_seed, "eval_seed": trainer.eval_seed,
            "n_gpus": world, "envs_per_gpu": trainer.E, "rollout_len": trainer.T, "algorithm": cfg.name}, indent=1))
    metrics_path = out / "training_metrics.jsonl"
    last: Dict[str, Any] = {}
    while trainer.iteration < cfg.num_iterations:
        t0 = time.perf_counter()
        res = trainer.train_iteration()
        if cfg.eval_interval and trainer.iteration % cfg.eval_interval == 0:
            res.update(trainer.evaluate())
        res["time_this_iter_s"] = time.perf_counter() - t0
        if rank == 0:
            with open(metrics_path, "a") as f:
                f.write(json.dumps(res) + "\n")
            ret = res.get("train/episode_return_mean")
            print(f"[iter {trainer.iteration:4d}] env_steps={res['num_env_steps_sampled_lifetime']} "
                  f"train_return={ret if ret is None else round(ret, 3)} "
                  f"eval_return={res.get('eval/episode_return_mean')} "
                  f"loss={res.get('learner/total_loss', float('nan')):.4f} ({res['time_this_iter_s']:.2f}s)",
                  flush=True)
        # every rank writes its own runtime state (env blob, generators); rank 0 the learner state
        if cfg.checkpoint_freq and trainer.iteration % cfg.checkpoint_freq == 0:
            trainer.save_checkpoint(out / "checkpoints" / f"checkpoint_{trainer.iteration:06d}")
        last = res
    trainer.save_checkpoint(out / "checkpoints" / "checkpoint_final")
    return last


def run_evaluate(args) -> Dict[str, Any]:
    from .ppo import PPOTrainer
    if not args.experiment_name:
        raise SystemExit("--experiment-name is required for --mode evaluate")
    out = Path(args.storage_dir) / args.experiment_name
    meta = json.loads((out / "run_metadata.json").read_text())
    env_cfg, algo_raw, cfg = _load_configs(str(out / "config_env.yaml"), str(out / "config_algorithm.yaml"))
    ckpt = Path(args.checkpoint) if args.checkpoint else out / "checkpoints" / "checkpoint_final"
    state = json.loads((ckpt / "state.json").read_text())
    env_meta = {}
    if state.get("obs_stats") is not None:
        import numpy as np
        env_meta["obs_stats"] = (np.asarray(state["obs_stats"][0], np.float32), np.asarray(state["obs_stats"][1], np.float32))
    root_seed = meta["root_seed"] if args.root_seed is None else args.root_seed
    trainer = PPOTrainer(env_cfg, cfg, root_seed=root_seed, n_envs=1, rollout_len=1,
                         device=0 if args.device is None else args.device, env_meta=env_meta, eval_seed=args.eval_seed)
    trainer.load_checkpoint(ckpt, runtime=False)  # weights only: evaluation builds its own envs
    n = args.eval_episodes or DEFAULT_EVAL_EPISODES
    res = trainer.evaluate(n)
    res.update({"checkpoint": str(ckpt), "root_seed": root_seed, "eval_seed": trainer.eval_seed,
                "iteration": trainer.iteration})
    (out / "eval_results.json").write_text(json.dumps(res, indent=1))
    print(json.dumps(res))
    return res


def main(argv: Optional[List[str]] = None) -> int:
    args = parse_args(argv)
    if args.mode == "single":
        run_single(args)
    else:
        run_evaluate(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
