"""On-device IPPO / MAPPO training: the RLlib PPO learner the reference configures, restated in
PyTorch-ROCm over the HIP env and the HIP GAE kernel.

Reference behaviour restated (RLlib 2.52.1 itself is not importable here: parity unpinned; the
tests check the loss against a direct restatement and the training loop's invariants):
* algorithm config: src/algorithms/ippo.py / mappo.py `_build_config` -- lr, train batch, epochs,
  minibatch = batch_size // num_minibatches, shuffled per epoch, clip_param, vf_clip_param,
  vf_loss_coeff, entropy_coeff, grad_clip (global norm), use_kl_loss, GAE(gamma, lambda);
  parameter sharing = one "shared_policy" module for every agent, else one module per agent
  (mappo.py:102-113), warehouse one-hot in the observation when sharing;
* loss: `PPOTorchLearner.compute_loss_for_module` -- clipped surrogate on exp(logp - logp_old),
  squared value error clipped at vf_clip_param, Gaussian entropy bonus, optional KL penalty with
  RLlib's adaptive coefficient (x1.5 above 2 kl_target, x0.5 below kl_target / 2);
* hysteretic weighting: src/algorithms/learners/hysteretic_learner.py:35-42 -- negative
  advantages scaled by hysteretic_beta before the loss;
* learning-rate schedules: [[timestep, lr], ...] piecewise linear in sampled env steps;
* observation statistics for meanstd_custom / meanstd_grouped: src/utils/obs_stats.py:11-169,
  the random-policy episodes run on the GPU env (same seeds, same action stream, bit-exact obs),
  the statistics on the host with numpy exactly as the reference computes them.

Multi-GPU: each rank steps its own env shard (global env ids, marlsc/dist.py), the advantage
statistics and the gradients (one flat f32 buffer per minibatch) are all-reduced -- RCCL over xGMI
on MI355X, gloo on CPU.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from .rollout import MLP, RolloutCollector, RolloutConfig, split_global_mlp

LOG2PI = math.log(2 * math.pi)
ENTROPY_CONST = 0.5 * math.log(2 * math.pi * math.e)


# ----------------------------------------------------------------------------------------------
# configuration (config_files/algorithms/*.yaml, schema.py SharedAlgorithmConfig / PPOConfig)
# ----------------------------------------------------------------------------------------------
@dataclass
class PPOConfig:
    name: str = "ippo"
    num_iterations: int = 100
    checkpoint_freq: int = 10
    batch_size: int = 4000
    num_epochs: int = 10
    num_minibatches: int = 4
    learning_rate: Union[float, List[List[float]]] = 5e-4
    num_env_runners: int = 0
    num_envs_per_env_runner: int = 1
    eval_interval: int = 1
    num_eval_episodes: int = 1
    use_gae: bool = True
    lam: float = 0.95
    gamma: float = 0.99
    use_kl_loss: bool = False
    kl_coeff: float = 0.2
    kl_target: float = 0.01
    grad_clip: Optional[float] = None
    entropy_coeff: float = 0.01
    vf_loss_coeff: float = 1.0
    clip_param: float = 0.2
    vf_clip_param: float = 10.0
    logstd_init: float = 0.0
    logstd_floor: float = -2.0
    obs_normalization: str = "off"
    parameter_sharing: bool = False
    hysteretic_beta: Optional[float] = None
    actor_obs_type: str = "local"
    critic_obs_type: str = "local"
    networks: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_algorithm_config(cls, cfg: Dict[str, Any]) -> "PPOConfig":
        a = cfg.get("algorithm", cfg)
        name = str(a.get("name", "ippo")).lower()
        if name not in ("ippo", "mappo"):
            raise ValueError(f"algorithm '{name}': this build trains ippo and mappo")
        sh = dict(a.get("shared", {}) or {})
        sp = dict(a.get("algorithm_specific", {}) or {})
        known = {f for f in cls.__dataclass_fields__}
        kw: Dict[str, Any] = {"name": name}
        for src in (sh, sp):
            for k, v in src.items():
                if k in known and v is not None:
                    kw[k] = v
        if "critic_obs_type" not in sp:
            kw["critic_obs_type"] = "global" if name == "mappo" else "local"
        c = cls(**kw)
        if c.lam < 0 or c.lam > 1 or c.gamma < 0 or c.gamma > 1:
            raise ValueError("lam and gamma must be in [0, 1]")
        if c.clip_param > 1.0:
            raise ValueError("clip_param should typically be <= 1.0")
        if c.hysteretic_beta is not None and not (0.0 < c.hysteretic_beta <= 1.0):
            raise ValueError("hysteretic_beta must be in (0.0, 1.0]")
        if c.obs_normalization == "meanstd":
            raise ValueError("obs_normalization 'meanstd' (RLlib's running MeanStdFilter connector) is not in this "
                             "build; use meanstd_custom / meanstd_grouped")
        return c

    def rollout_config(self) -> RolloutConfig:
        nets = self.networks or {}
        if nets.get("shared_layers"):
            raise ValueError("shared_layers (GRU) networks are outside this build's training path")
        return RolloutConfig(gamma=float(self.gamma), lam=float(self.lam) if self.use_gae else 1.0,
                             actor_obs_type=self.actor_obs_type, critic_obs_type=self.critic_obs_type,
                             logstd_init=float(self.logstd_init), logstd_floor=float(self.logstd_floor),
                             actor=(nets.get("actor") or {}).get("config"),
                             critic=(nets.get("critic") or {}).get("config"))

    def lr_at(self, timestep: int) -> float:
        """RLlib learning-rate schedule: piecewise linear over [[t, lr], ...], constant outside."""
        lr = self.learning_rate
        if isinstance(lr, (int, float)):
            return float(lr)
        pts = sorted((float(t), float(v)) for t, v in lr)
        if timestep <= pts[0][0]:
            return pts[0][1]
        for (t0, v0), (t1, v1) in zip(pts, pts[1:]):
            if timestep < t1:
                return v0 + (v1 - v0) * (timestep - t0) / (t1 - t0)
        return pts[-1][1]


# ----------------------------------------------------------------------------------------------
# modules: one shared policy or one per agent (the reference's policy mapping, mappo.py:102-113)
# ----------------------------------------------------------------------------------------------
class AgentModule(nn.Module):
    """ActorCriticRLModule for MLP networks (rlmodules/base.py:480-715)."""

    def __init__(self, local_obs_dim: int, global_obs_dim: int, action_dim: int, rc: RolloutConfig):
        super().__init__()
        full = local_obs_dim + global_obs_dim
        self.actor = MLP(full if rc.actor_obs_type == "global" else local_obs_dim, action_dim,
                         rc.actor or {"hidden_sizes": [256, 256]})
        self.critic = MLP(full if rc.critic_obs_type == "global" else local_obs_dim, 1,
                          rc.critic or {"hidden_sizes": [256, 256]})
        self.log_std = nn.Parameter(torch.full((action_dim,), float(rc.logstd_init)))


class MultiAgentActorCritic(nn.Module):
    """dist_inputs / values over [..., W, obs] for the shared policy or W per-agent policies."""

    def __init__(self, n_agents: int, local_obs_dim: int, global_obs_dim: int, action_dim: int, rc: RolloutConfig,
                 shared: bool):
        super().__init__()
        self.rc, self.shared, self.W = rc, bool(shared), int(n_agents)
        self.policies = nn.ModuleList([AgentModule(local_obs_dim, global_obs_dim, action_dim, rc)
                                       for _ in range(1 if shared else n_agents)])

    def _x(self, local_obs, full_obs, kind):
        return full_obs if kind == "global" else local_obs

    def _per_agent(self, fn, x):
        if self.shared:
            return fn(self.policies[0], x)
        return torch.stack([fn(p, x[..., w, :]) for w, p in enumerate(self.policies)], dim=-2)

    def dist_inputs(self, local_obs, full_obs=None):
        x = self._x(local_obs, full_obs, self.rc.actor_obs_type)
        floor = self.rc.logstd_floor
        mean = self._per_agent(lambda p, v: p.actor(v), x)
        if self.shared:
            log_std = torch.clamp(self.policies[0].log_std, min=floor).expand_as(mean)
        else:
            log_std = torch.stack([torch.clamp(p.log_std, min=floor) for p in self.policies])  # [W, K]
            log_std = log_std.expand_as(mean)
        return mean, log_std

    def values(self, local_obs, full_obs=None):
        if self.rc.critic_obs_type == "global" and full_obs is None:  # split first layer (rollout.py)
            if self.shared:
                return split_global_mlp(self.policies[0].critic, local_obs).squeeze(-1)
            return torch.stack([split_global_mlp(p.critic, local_obs, w).squeeze(-1)
                                for w, p in enumerate(self.policies)], dim=-1)
        x = self._x(local_obs, full_obs, self.rc.critic_obs_type)
        if self.shared:
            return self.policies[0].critic(x).squeeze(-1)
        return torch.stack([p.critic(x[..., w, :]).squeeze(-1) for w, p in enumerate(self.policies)], dim=-1)


def gaussian_logp(a: torch.Tensor, mean: torch.Tensor, log_std: torch.Tensor) -> torch.Tensor:
    std = log_std.exp()
    return (-((a - mean) ** 2) / (2 * std * std) - log_std - 0.5 * LOG2PI).sum(-1)


def gaussian_entropy(log_std: torch.Tensor) -> torch.Tensor:
    return (log_std + ENTROPY_CONST).sum(-1)


def gaussian_kl(mean0, log_std0, mean1, log_std1) -> torch.Tensor:
    """KL(old || new) of diagonal Gaussians (RLlib TorchDiagGaussian.kl)."""
    v0, v1 = (2 * log_std0).exp(), (2 * log_std1).exp()
    return (log_std1 - log_std0 + (v0 + (mean0 - mean1) ** 2) / (2 * v1) - 0.5).sum(-1)


def ppo_loss(cfg: PPOConfig, mean, log_std, values, batch: Dict[str, torch.Tensor], kl_coeff: float):
    """PPOTorchLearner.compute_loss_for_module (with the hysteretic advantage weighting)."""
    adv = batch["advantages"]
    if cfg.hysteretic_beta is not None and cfg.hysteretic_beta < 1.0:
        adv = adv * torch.where(adv >= 0, torch.ones_like(adv), torch.full_like(adv, cfg.hysteretic_beta))
    logp = gaussian_logp(batch["actions"], mean, log_std)
    ratio = torch.exp(logp - batch["logp"])
    surrogate = torch.minimum(adv * ratio, adv * torch.clamp(ratio, 1 - cfg.clip_param, 1 + cfg.clip_param))
    entropy = gaussian_entropy(log_std)
    vf_loss = (values - batch["value_targets"]) ** 2
    vf_clipped = torch.clamp(vf_loss, 0, cfg.vf_clip_param)
    total = (-surrogate + cfg.vf_loss_coeff * vf_clipped - cfg.entropy_coeff * entropy).mean()
    stats = {"policy_loss": -surrogate.mean(), "vf_loss": vf_clipped.mean(), "entropy": entropy.mean()}
    if cfg.use_kl_loss:
        kl = gaussian_kl(batch["mean_old"], batch["log_std_old"], mean, log_std).mean()
        total = total + kl_coeff * kl
        stats["mean_kl"] = kl
    stats["total_loss"] = total
    return total, stats


def allreduce_grads(params: Sequence[nn.Parameter]) -> None:
    """Average gradients over ranks: one flat buffer, one all-reduce (RCCL / gloo)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat /= dist.get_world_size()
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


class PPOLearner:
    """Minibatch SGD over one collected batch (num_epochs x num_minibatches, shuffled per epoch)."""

    def __init__(self, module: MultiAgentActorCritic, cfg: PPOConfig, *, seed: int = 0):
        self.module, self.cfg = module, cfg
        self.opt = torch.optim.Adam(module.parameters(), lr=cfg.lr_at(0))
        self.kl_coeff = float(cfg.kl_coeff)
        dev = next(module.parameters()).device
        self.gen = torch.Generator(device=dev).manual_seed(int(seed))

    def update(self, batch: Dict[str, torch.Tensor], full_fn, timestep: int) -> Dict[str, float]:
        """batch tensors are [S, W, ...] (S = samples of one agent slot); full_fn(obs) -> flat obs."""
        cfg, m = self.cfg, self.module
        for g in self.opt.param_groups:
            g["lr"] = cfg.lr_at(timestep)
        S = batch["obs"].shape[0]
        mb = max(1, S // max(1, cfg.num_minibatches))
        acc: Dict[str, float] = {}
        n = 0
        for _ in range(cfg.num_epochs):
            perm = torch.randperm(S, device=batch["obs"].device, generator=self.gen)
            for i in range(0, S - mb + 1, mb):
                idx = perm[i:i + mb]
                b = {k: v[idx] for k, v in batch.items()}
                full = full_fn(b["obs"]) if full_fn is not None else None
                mean, log_std = m.dist_inputs(b["obs"], full)
                values = m.values(b["obs"], full)
                loss, st = ppo_loss(cfg, mean, log_std, values, b, self.kl_coeff)
                self.opt.zero_grad(set_to_none=True)
                loss.backward()
                params = [p for p in m.parameters() if p.grad is not None]
                allreduce_grads(params)
                if cfg.grad_clip:
                    torch.nn.utils.clip_grad_norm_(params, cfg.grad_clip)
                self.opt.step()
                for k, v in st.items():
                    acc[k] = acc.get(k, 0.0) + float(v.detach())
                n += 1
        out = {k: v / max(n, 1) for k, v in acc.items()}
        if cfg.use_kl_loss and "mean_kl" in out:  # RLlib's adaptive KL coefficient
            if out["mean_kl"] > 2.0 * cfg.kl_target:
                self.kl_coeff *= 1.5
            elif out["mean_kl"] < 0.5 * cfg.kl_target:
                self.kl_coeff *= 0.5
            out["kl_coeff"] = self.kl_coeff
        out["learning_rate"] = self.opt.param_groups[0]["lr"]
        return out


# ----------------------------------------------------------------------------------------------
# observation statistics (src/utils/obs_stats.py:11-169) on the GPU env
# ----------------------------------------------------------------------------------------------
def feature_groups(spec) -> List[Tuple[int, bool]]:
    """(per-SKU column count, has aggregate) per enabled group, obs_stats.py:_compute_grouped_stats."""
    f, K = spec.features, spec.K
    g: List[Tuple[int, bool]] = []
    if f.get("inventory"):
        g.append((K, bool(f.get("inventory_aggregate"))))
    if f.get("pipeline"):
        g.append((spec.max_expected_lead_time * K, bool(f.get("pipeline_aggregate"))))
    if f.get("incoming_demand_home"):
        g.append((K, bool(f.get("incoming_demand_home_aggregate"))))
    if f.get("units_shipped_home"):
        g.append((K, False))
    if f.get("units_shipped_away"):
        g.append((K, bool(f.get("units_shipped_away_aggregate"))))
    if f.get("stockout"):
        g.append((K, False))
    if f.get("rolling_demand_mean"):
        g.append((K, bool(f.get("rolling_demand_mean_aggregate"))))
    if f.get("demand_forecast"):
        g.append((K, bool(f.get("demand_forecast_aggregate"))))
    return g


def obs_statistics_from_samples(all_obs: np.ndarray, mode: str, spec=None) -> Tuple[np.ndarray, np.ndarray]:
    """numpy statistics exactly as the reference computes them from its collected f32 samples."""
    all_obs = np.asarray(all_obs, dtype=np.float32)
    if mode == "meanstd_grouped":
        dim = all_obs.shape[1]
        mean = np.zeros(dim, dtype=np.float32)
        std = np.ones(dim, dtype=np.float32)
        idx = 0
        for cnt, agg in feature_groups(spec):
            blk = all_obs[:, idx:idx + cnt]
            mean[idx:idx + cnt] = float(blk.mean())
            std[idx:idx + cnt] = float(blk.std())
            idx += cnt
            if agg:
                col = all_obs[:, idx]
                mean[idx] = float(col.mean())
                std[idx] = float(col.std())
                idx += 1
    else:
        mean = all_obs.mean(axis=0)
        std = all_obs.std(axis=0)
    std = np.where(std < 1e-8, 1.0, std)
    return mean, std


def compute_obs_statistics(env_config: Any, seed_manager, mode: str = "meanstd_custom", n_episodes: int = 10,
                           device: int = 0, env_meta: Optional[Dict[str, Any]] = None):
    """compute_obs_statistics (obs_stats.py:11-90): a random policy for n_episodes on ONE env seeded
    with the first 'obs_stats' child seed (its episodes re-seed through SeedManager.advance_episode,
    as the reference's sequential resets do), actions uniform[-1, 1] f32 from the second child seed
    in agent order; the env runs on the GPU, the statistics on the host."""
    from .spec import EnvSpec
    from .vec_env import VecInventoryEnv
    env_seed, action_seed = seed_manager.spawn_child_seeds("obs_stats", 2)
    meta = dict(env_meta or {})
    meta.pop("include_warehouse_id", None)
    meta["obs_normalization"] = "off"
    meta.pop("obs_stats", None)
    spec = EnvSpec.from_config(env_config, meta)
    env = VecInventoryEnv(None, 1, spec=spec, device=device, env_seeds=np.array([env_seed], dtype=np.uint32))
    rng = np.random.default_rng(action_seed)
    W, K, T = spec.W, spec.K, spec.episode_length
    samples = []
    obs = env.reset()
    for _ in range(n_episodes):
        for t in range(T):
            samples.append(obs[0].cpu().numpy())
            a = np.stack([rng.uniform(-1, 1, size=(K,)).astype(np.float32) for _ in range(W)])
            obs, _, trunc, final = env.step(torch.from_numpy(a).to(env.device).unsqueeze(0))
        samples.append(final[0].cpu().numpy())  # the terminal observation of the episode
    env.close()
    all_obs = np.concatenate(samples, axis=0)  # [(T + 1) * n_episodes * W, L] in agent order
    return obs_statistics_from_samples(all_obs, mode, spec)


# ----------------------------------------------------------------------------------------------
# trainer (ExperimentRunner.run, src/experiments/runner.py)
# ----------------------------------------------------------------------------------------------
class PPOTrainer:
    def __init__(self, env_config: Any, cfg: PPOConfig, *, root_seed: int = 42, n_envs: Optional[int] = None,
                 rollout_len: Optional[int] = None, device: int = 0, env_meta: Optional[Dict[str, Any]] = None,
                 eval_seed: Optional[int] = None):
        from .seeding import SeedManager
        from .spec import EnvSpec
        from .vec_env import VecInventoryEnv
        self.cfg = cfg
        self.rank, self.world = (dist.get_rank(), dist.get_world_size()) if (dist.is_available() and dist.is_initialized()) else (0, 1)
        self.root_seed = int(root_seed)
        self.sm = SeedManager(self.root_seed)
        self.train_seed = self.sm.get_seed_int("train")
        self.eval_seed = eval_seed if eval_seed is not None else self.sm.get_seed_int("eval")
        meta = dict(env_meta or {})
        meta["include_warehouse_id"] = bool(cfg.parameter_sharing)
        meta["obs_normalization"] = cfg.obs_normalization
        if cfg.obs_normalization in ("meanstd_custom", "meanstd_grouped") and meta.get("obs_stats") is None:
            meta["obs_stats"] = compute_obs_statistics(env_config, self.sm, cfg.obs_normalization, n_episodes=100,
                                                       device=device, env_meta=meta)
        self.env_meta = meta
        self.env_config = env_config
        self.spec = EnvSpec.from_config(env_config, meta)
        E = int(n_envs or max(1, cfg.num_envs_per_env_runner) * max(1, cfg.num_env_runners))
        self.E = E
        # rollout length: RLlib's train batch counts env steps over every runner of every rank
        self.T = int(rollout_len or max(1, math.ceil(cfg.batch_size / (E * self.world))))
        self.device = torch.device("cuda", device)
        self.env = VecInventoryEnv(None, E, spec=self.spec, device=device, base_seed=self.train_seed,
                                   env_index_offset=self.rank * E)
        rc = cfg.rollout_config()
        torch.manual_seed(self.train_seed)
        W, L = self.env.W, self.env.local_obs_dim
        self.module = MultiAgentActorCritic(W, L, L * W, self.env.K, rc, cfg.parameter_sharing).to(self.device)
        if self.world > 1:  # identical initial weights on every rank
            for p in self.module.parameters():
                dist.broadcast(p.data, src=0)
        self.learner = PPOLearner(self.module, cfg, seed=self.train_seed + self.rank)
        self.collector = RolloutCollector(self.env, self.module, self.T, seed=self.train_seed + 1000 + self.rank)
        self.env.reset()
        self.iteration = 0
        self.timesteps = 0
        self._ep_ret = torch.zeros(E, dtype=torch.float64, device=self.device)
        self._completed: List[float] = []

    def _full_fn(self):
        if self.cfg.actor_obs_type != "global":  # the critic evaluates its split first layer
            return None
        W, L = self.env.W, self.env.local_obs_dim

        def full(obs):  # obs [S, W, L] of S whole envs -> local || global per agent
            g = obs.reshape(obs.shape[0], 1, W * L).expand(obs.shape[0], W, W * L)
            return torch.cat([obs, g], dim=-1)
        return full

    def train_iteration(self) -> Dict[str, Any]:
        cfg, T, E, W = self.cfg, self.T, self.E, self.env.W
        out = self.collector.collect(normalize=True)
        # episode returns (sum over agents, RLlib's multi-agent episode return)
        rew = self.collector.rewards.double().sum(-1)  # [T, E]
        trunc = self.collector.truncated[:, :, 0].bool()
        for t in range(T):
            self._ep_ret += rew[t]
            if bool(trunc[t].any()):
                self._completed.extend(self._ep_ret[trunc[t]].tolist())
                self._ep_ret[trunc[t]] = 0.0
        self.timesteps += T * E * self.world
        batch = {"obs": out["obs"].reshape(T * E, W, -1), "actions": out["actions"].reshape(T * E, W, -1),
                 "logp": out["logp"].reshape(T * E, W), "advantages": out["advantages"].reshape(T * E, W),
                 "value_targets": out["value_targets"].reshape(T * E, W)}
        if cfg.use_kl_loss:
            with torch.no_grad():
                mo, lo = self.module.dist_inputs(batch["obs"], self._full_fn()(batch["obs"]) if self._full_fn() else None)
            batch["mean_old"], batch["log_std_old"] = mo, lo
        stats = self.learner.update(batch, self._full_fn(), self.timesteps)
        self.iteration += 1
        done = self._completed[-max(1, cfg.num_eval_episodes) * E:]
        res = {"training_iteration": self.iteration, "num_env_steps_sampled_lifetime": self.timesteps,
               "train/episode_return_mean": float(np.mean(done)) if done else None,
               "train/episodes": len(self._completed)}
        res.update({f"learner/{k}": v for k, v in stats.items()})
        return res

    @torch.no_grad()
    def evaluate(self, n_episodes: Optional[int] = None, seed: Optional[int] = None) -> Dict[str, Any]:
        """Deterministic (mean-action) episodes on fresh eval envs ('val' data mode)."""
        from .spec import EnvSpec
        from .vec_env import VecInventoryEnv
        n = int(n_episodes or self.cfg.num_eval_episodes)
        meta = dict(self.env_meta)
        meta["data_mode"] = "val"
        spec = EnvSpec.from_config(self.env_config, meta)
        env = VecInventoryEnv(None, n, spec=spec, device=self.device.index,
                              base_seed=self.eval_seed if seed is None else int(seed))
        obs = env.reset()
        full_fn = self._full_fn()
        ret = torch.zeros(n, dtype=torch.float64, device=self.device)
        for _ in range(spec.episode_length):
            full = env.obs_flat(obs=obs) if full_fn is not None else None
            mean, _ = self.module.dist_inputs(obs, full)
            obs, rew, trunc, _ = env.step(mean.clamp(-1.0, 1.0).contiguous())
            ret += rew.double().sum(-1)
        env.close()
        r = ret.cpu().numpy()
        return {"eval/episode_return_mean": float(r.mean()), "eval/episode_return_std": float(r.std()),
                "eval/episodes": n}

    # -- checkpoints (module + optimizer + counters + configs) --------------------------------
    def save_checkpoint(self, path: Union[str, Path]) -> Path:
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        torch.save({"module": self.module.state_dict(), "optimizer": self.learner.opt.state_dict(),
                    "kl_coeff": self.learner.kl_coeff, "iteration": self.iteration, "timesteps": self.timesteps},
                   p / "learner_state.pt")
        stats = self.env_meta.get("obs_stats")
        (p / "state.json").write_text(json.dumps({
            "iteration": self.iteration, "timesteps": self.timesteps, "root_seed": self.root_seed,
            "algorithm": asdict(self.cfg),
            "obs_stats": None if stats is None else [np.asarray(stats[0]).tolist(), np.asarray(stats[1]).tolist()]},
            indent=1))
        return p

    def load_checkpoint(self, path: Union[str, Path]) -> None:
        st = torch.load(Path(path) / "learner_state.pt", map_location=self.device, weights_only=True)
        self.module.load_state_dict(st["module"])
        self.learner.opt.load_state_dict(st["optimizer"])
        self.learner.kl_coeff = float(st["kl_coeff"])
        self.iteration = int(st["iteration"])
        self.timesteps = int(st["timesteps"])
