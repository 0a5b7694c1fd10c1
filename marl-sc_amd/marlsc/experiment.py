"""CLI of the reference's experiment entry point (src/experiments/run_experiment.py), for the modes
that drive this build's training path: `single` (train one seed, with periodic evaluation and
checkpoints) and `evaluate` (deterministic episodes from a checkpoint). Ray Tune sweeps, seed
evaluation and W&B are out of scope; their flags are accepted and ignored.

    python -m marlsc.experiment --mode single --env-config ENV.yaml --algorithm-config ALGO.yaml \
        --storage-dir ./experiment_outputs --experiment-name NAME --root-seed 42
    python -m marlsc.experiment --mode evaluate --storage-dir ./experiment_outputs \
        --experiment-name NAME --eval-episodes 100 --root-seed 42

Multi-GPU: launch `single` with torchrun (one process per GPU, RCCL; MSC_DIST_BACKEND=gloo
rehearses it on CPU-side collectives); each rank owns `--envs` envs (global env ids), gradients and
advantage statistics are all-reduced.
Output layout (per experiment directory, as the reference's ExperimentRunner writes it,
src/experiments/runner.py:163-395): checkpoint_<N>/ every checkpoint_freq iterations,
checkpoint_best/ on each new best train return, checkpoint_final/, module_weights.pt (the state
dict of agent 0's policy module, src/utils/weight_transfer.py:15-33), training_metrics.yaml
({iteration, train_return, eval_return} per iteration; truncated to N on --resume-from
checkpoint_<N>, runner.py:231-288), metadata.json, config_env.yaml, config_algorithm.yaml; plus
training_metrics.jsonl (every result key per iteration) and eval_results.json (evaluate mode).
"""
from __future__ import annotations

import argparse
import json
import os
import re
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
    """One process per GPU (torchrun env). Backend: MSC_DIST_BACKEND (default nccl = RCCL on ROCm;
    gloo rehearses the multi-rank path, e.g. several ranks sharing one GPU)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("MSC_DIST_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count()) if torch.cuda.is_available() else 0
        if torch.cuda.is_available():
            torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        local = dev
    return (dist.get_rank() if world > 1 else 0), world, local


# ---- run-directory bookkeeping of the reference runner (src/experiments/runner.py,
# ---- src/experiments/utils/experiment_utils.py:256-467)
_CKPT_RE = re.compile(r"^checkpoint_(\d+)$")


def parse_checkpoint_iteration(path) -> Optional[int]:
    """N of a checkpoint_<N> directory; None for checkpoint_best / checkpoint_final."""
    m = _CKPT_RE.match(Path(path).name)
    return int(m.group(1)) if m else None


def save_training_metrics(out: Path, metrics: List[Dict[str, Any]]) -> None:
    with open(out / "training_metrics.yaml", "w", encoding="utf-8") as f:
        yaml.dump(metrics, f, default_flow_style=False, sort_keys=False)


def load_and_truncate_training_metrics(out: Path, completed: int):
    """training_metrics.yaml entries with iteration <= completed, and the best train return among
    them (-inf / None when there is none)."""
    metrics: List[Dict[str, Any]] = []
    path = out / "training_metrics.yaml"
    if path.exists():
        existing = yaml.safe_load(path.read_text()) or []
        if isinstance(existing, list):
            metrics = [m for m in existing if isinstance(m, dict) and isinstance(m.get("iteration"), int)
                       and m["iteration"] <= completed]
    best, best_it = float("-inf"), None
    for m in metrics:
        tr = m.get("train_return")
        if isinstance(tr, (int, float)) and tr > best:
            best, best_it = float(tr), m["iteration"]
    return metrics, best, best_it


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
    metrics: List[Dict[str, Any]] = []
    best, best_it = float("-inf"), None
    if args.resume_from:
        # runner.py:231-288: resume from checkpoint_<N>, metrics truncated to N, best restored
        completed = parse_checkpoint_iteration(args.resume_from)
        if completed is None:
            raise ValueError("--resume-from must point at a 'checkpoint_<N>' directory so training can continue "
                             f"from iteration N+1. Got: {args.resume_from}")
        trainer.load_checkpoint(args.resume_from)
        if trainer.iteration != completed:
            raise ValueError(f"{args.resume_from} holds iteration {trainer.iteration}, not {completed}")
        metrics, best, best_it = load_and_truncate_training_metrics(out, completed)
    if rank == 0:
        out.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(args.env_config, out / "config_env.yaml")
        shutil.copyfile(args.algorithm_config, out / "config_algorithm.yaml")
        meta = out / "metadata.json"
        if not meta.exists():  # written once per run (experiment_utils.save_run_metadata)
            meta.write_text(json.dumps({
                "root_seed": root_seed, "train_seed": trainer.train_seed, "eval_seed": trainer.eval_seed,
                "n_gpus": world, "envs_per_gpu": trainer.E, "rollout_len": trainer.T, "algorithm": cfg.name}, indent=1))
        if args.resume_from:  # the detailed log is truncated like the yaml one
            jl = out / "training_metrics.jsonl"
            if jl.exists():
                keep = [ln for ln in jl.read_text().splitlines()
                        if ln.strip() and json.loads(ln).get("training_iteration", 0) <= trainer.iteration]
                jl.write_text("".join(k + "\n" for k in keep))
    last: Dict[str, Any] = {}
    while trainer.iteration < cfg.num_iterations:
        t0 = time.perf_counter()
        res = trainer.train_iteration()
        it = trainer.iteration
        if cfg.eval_interval and it % cfg.eval_interval == 0:
            res.update(trainer.evaluate())
        res["time_this_iter_s"] = time.perf_counter() - t0
        train_ret = res.get("train/episode_return_mean")
        metrics.append({"iteration": it, "train_return": train_ret, "eval_return": res.get("eval/episode_return_mean")})
        # checkpoint_best on a strictly better train return (runner.py:290-339); every rank saves its
        # runtime state into the same directory, rank 0 the learner state. The return is all-reduced
        # (PPOTrainer._global_train_return) and rank 0's decision is broadcast, so every rank takes the
        # same branch (the barrier and the save are collective across ranks)
        new_best = _agree(train_ret is not None and train_ret > best, world)
        if new_best:
            best, best_it = float(train_ret), it
            bp = out / "checkpoint_best"
            if rank == 0 and bp.exists():
                shutil.rmtree(bp)
            _barrier(world)
            trainer.save_checkpoint(bp)
        if rank == 0:
            save_training_metrics(out, metrics)
            with open(out / "training_metrics.jsonl", "a") as f:
                f.write(json.dumps(res) + "\n")
            print(f"[iter {it:4d}] env_steps={res['num_env_steps_sampled_lifetime']} "
                  f"train_return={train_ret if train_ret is None else round(train_ret, 3)} "
                  f"eval_return={res.get('eval/episode_return_mean')} "
                  f"loss={res.get('learner/total_loss', float('nan')):.4f} ({res['time_this_iter_s']:.2f}s)",
                  flush=True)
        if cfg.checkpoint_freq and it % cfg.checkpoint_freq == 0:
            trainer.save_checkpoint(out / f"checkpoint_{it}")
        last = res
    if rank == 0 and best_it is not None:
        print(f"[INFO] Best checkpoint: iteration {best_it} with reward: {best:.4f}")
    trainer.save_checkpoint(out / "checkpoint_final")
    if rank == 0:
        trainer.export_module_weights(out / "module_weights.pt")
        if metrics:
            save_training_metrics(out, metrics)
    return last


def _agree(flag: bool, world: int) -> bool:
    """Rank 0's value of `flag` on every rank."""
    if world <= 1:
        return bool(flag)
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.broadcast(t, src=0)
    return bool(int(t.item()))


def _barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def run_evaluate(args) -> Dict[str, Any]:
    from .ppo import PPOTrainer
    if not args.experiment_name:
        raise SystemExit("--experiment-name is required for --mode evaluate")
    out = Path(args.storage_dir) / args.experiment_name
    mp = out / "metadata.json"
    meta = json.loads((mp if mp.exists() else out / "run_metadata.json").read_text())
    env_cfg, algo_raw, cfg = _load_configs(str(out / "config_env.yaml"), str(out / "config_algorithm.yaml"))
    ckpt = Path(args.checkpoint) if args.checkpoint else out / "checkpoint_final"
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
