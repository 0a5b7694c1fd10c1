"""On-device IPPO / MAPPO training: the RLlib PPO learner the reference configures, restated in
PyTorch-ROCm over the HIP env and the HIP GAE kernel.

Reference behaviour restated (RLlib 2.52.1 itself is not importable here: parity unpinned; the
tests check the loss against a direct restatement and the training loop's invariants):
* algorithm config: src/algorithms/ippo.py / mappo.py `_build_config` -- lr, train batch, epochs,
  minibatch_size = batch_size // num_minibatches (mappo.py:148), shuffled per epoch, clip_param,
  vf_clip_param, vf_loss_coeff, entropy_coeff, grad_clip (global norm), use_kl_loss,
  GAE(gamma, lambda); parameter sharing = one "shared_policy" module for every agent, else one
  module per agent (mappo.py:102-113), warehouse one-hot in the observation when sharing;
* minibatches: RLlib's MiniBatchCyclicIterator -- every module's batch (its AGENT steps: all
  W agents' rows for the shared policy, one agent's rows per per-agent policy) is cut into
  minibatches of minibatch_size rows, cycling through reshuffled epochs until every module has
  covered num_epochs passes; one optimizer step per minibatch over every module at once. The
  shared policy of W agents therefore takes W x num_minibatches steps per epoch;
* loss: `PPOTorchLearner.compute_loss_for_module` per module -- clipped surrogate on
  exp(logp - logp_old), squared value error clipped at vf_clip_param, Gaussian entropy bonus,
  optional KL penalty with RLlib's adaptive coefficient (x1.5 above 2 kl_target, x0.5 below
  kl_target / 2); the learner minimises the SUM of the module losses and clips each module's
  gradients by its own global norm (TorchLearner.compute_gradients / postprocess_gradients);
* advantages are standardised per module (RLlib's GAE connector): over all agents for the shared
  policy, per agent otherwise (marlsc/rollout.py, msc_gae_grouped);
* hysteretic weighting: src/algorithms/learners/hysteretic_learner.py:35-42 -- negative
  advantages scaled by hysteretic_beta before the loss;
* learning-rate schedules: [[timestep, lr], ...] piecewise linear in sampled env steps;
* observation statistics for meanstd_custom / meanstd_grouped: src/utils/obs_stats.py:11-169,
  the random-policy episodes run on the GPU env (same seeds, same action stream, bit-exact obs),
  the statistics on the host with numpy exactly as the reference computes them;
* obs_normalization "meanstd": RLlib's running MeanStdFilter connector (mappo.py:170-171) on the
  device, synchronised after every rollout and applied with update=False in evaluation
  (base.py:131-140; marlsc/obs_filter.py).

Multi-GPU: each rank steps its own env shard (global env ids, marlsc/dist.py), the advantage
statistics and the gradients (one flat f32 buffer per minibatch) are all-reduced -- RCCL over xGMI
on MI355X, gloo on CPU.
"""
from __future__ import annotations

import json
import math
import os
import warnings
from collections import deque
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import dist as mdist
from .rollout import MLP, RolloutCollector, RolloutConfig, fused_actor_sample, mlp_forward, split_global_mlp

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
        if c.obs_normalization not in ("off", "ratio", "meanstd", "meanstd_custom", "meanstd_grouped"):
            raise ValueError(f"obs_normalization '{c.obs_normalization}' is not one of off / ratio / meanstd / "
                             "meanstd_custom / meanstd_grouped")
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

    def actor_mean(self, local_obs, full_obs=None):
        return self._per_agent(lambda p, v: p.actor(v), self._x(local_obs, full_obs, self.rc.actor_obs_type))

    def log_std_table(self) -> torch.Tensor:
        """[P, K] unclamped log_std rows (P = 1 shared, W per agent) for msc_gaussian_sample, which
        applies logstd_floor itself."""
        return torch.stack([p.log_std.detach().float() for p in self.policies]).contiguous()

    def actor_sample(self, local_obs, full_obs, sample) -> bool:
        """Shared policy: the actor with the rollout's action sampling fused into its kernel."""
        if not self.shared:
            return False
        return fused_actor_sample(self.policies[0].actor, self._x(local_obs, full_obs, self.rc.actor_obs_type), sample)

    def dist_inputs(self, local_obs, full_obs=None):
        floor = self.rc.logstd_floor
        mean = self.actor_mean(local_obs, full_obs)
        if self.shared:
            log_std = torch.clamp(self.policies[0].log_std, min=floor).expand_as(mean)
        else:
            log_std = torch.stack([torch.clamp(p.log_std, min=floor) for p in self.policies])  # [W, K]
            log_std = log_std.expand_as(mean)
        return mean, log_std

    def values(self, local_obs, full_obs=None, out=None):
        if self.rc.critic_obs_type == "global" and full_obs is None:  # split first layer (rollout.py)
            if self.shared:
                return split_global_mlp(self.policies[0].critic, local_obs, out=out).squeeze(-1)
            return torch.stack([split_global_mlp(p.critic, local_obs, w).squeeze(-1)
                                for w, p in enumerate(self.policies)], dim=-1)
        x = self._x(local_obs, full_obs, self.rc.critic_obs_type)
        if self.shared:
            return mlp_forward(self.policies[0].critic, x, out=out).squeeze(-1)
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


class _CyclicRows:
    """One module's row stream of RLlib's MiniBatchCyclicIterator: minibatches of `mb` rows cut from
    a shuffled pass over the module's M rows, wrapping into the next (reshuffled) pass; `covered`
    counts the passes completed."""

    def __init__(self, rows: torch.Tensor, mb: int, gen: torch.Generator):
        self.rows, self.mb, self.gen = rows, int(mb), gen
        self.M = rows.numel()
        self.start, self.covered = 0, 0
        self.perm = self._shuffle()

    def _shuffle(self) -> torch.Tensor:
        return self.rows[torch.randperm(self.M, device=self.rows.device, generator=self.gen)]

    def next(self) -> torch.Tensor:
        parts, start, stop = [], self.start, self.start + self.mb
        while stop >= self.M:
            parts.append(self.perm[start:])
            self.covered += 1
            self.perm = self._shuffle()
            stop -= self.M
            start = 0
        parts.append(self.perm[start:stop])
        self.start = stop
        return torch.cat(parts) if len(parts) > 1 else parts[0]


def minibatch_rows(cfg: "PPOConfig", world: int = 1) -> int:
    """Rows per module and minibatch on one rank: RLlib's minibatch_size = batch_size //
    num_minibatches agent steps per module (mappo.py:148), split over the ranks that all-reduce
    their gradients (each rank holds 1/world of the train batch)."""
    mb = max(1, int(cfg.batch_size) // max(1, int(cfg.num_minibatches)))
    return max(1, mb // max(1, int(world)))


class PPOLearner:
    """Minibatch SGD over one collected batch, module by module as RLlib's learner does."""

    @property
    def kl_coeff(self) -> float:
        return float(np.mean(self.kl_coeffs))

    def __init__(self, module: MultiAgentActorCritic, cfg: PPOConfig, *, seed: int = 0):
        self.module, self.cfg = module, cfg
        self.opt = torch.optim.Adam(module.parameters(), lr=cfg.lr_at(0))
        # RLlib keeps one adaptive KL coefficient per module
        self.kl_coeffs = [float(cfg.kl_coeff)] * len(module.policies)
        dev = next(module.parameters()).device
        self.gen = torch.Generator(device=dev).manual_seed(int(seed))
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1

    def _module_rows(self, S: int, W: int, device) -> List[torch.Tensor]:
        """Flat row ids (s * W + w) of every module's batch: all rows for the shared policy, agent
        w's rows for policy w."""
        if self.module.shared:
            return [torch.arange(S * W, device=device)]
        return [torch.arange(S, device=device) * W + w for w in range(W)]

    def _forward(self, policy: "AgentModule", obs: torch.Tensor, rows: torch.Tensor):
        """(mean, log_std, values) of `policy` on batch rows (flat ids s * W + w of obs [S, W, L])."""
        rc = self.module.rc
        S, W, L = obs.shape
        local = obs.reshape(S * W, L)[rows]
        full = None
        if rc.actor_obs_type == "global" or rc.critic_obs_type == "global":
            full = torch.cat([local, obs[torch.div(rows, W, rounding_mode="floor")].reshape(-1, W * L)], dim=-1)
        mean = policy.actor(full if rc.actor_obs_type == "global" else local)
        log_std = torch.clamp(policy.log_std, min=rc.logstd_floor).expand_as(mean)
        values = policy.critic(full if rc.critic_obs_type == "global" else local).squeeze(-1)
        return mean, log_std, values

    def update(self, batch: Dict[str, torch.Tensor], full_fn=None, timestep: int = 0) -> Dict[str, float]:
        """batch tensors are [S, W, ...] (S env samples of W agents). full_fn is unused (the learner
        gathers each row's local || global observation itself) and kept for call compatibility."""
        cfg, m = self.cfg, self.module
        for g in self.opt.param_groups:
            g["lr"] = cfg.lr_at(timestep)
        obs = batch["obs"]
        S, W = obs.shape[0], obs.shape[1]
        flat = {k: v.reshape(S * W, *v.shape[2:]) for k, v in batch.items() if k != "obs"}
        mb = minibatch_rows(cfg, self.world)
        streams = [_CyclicRows(r, min(mb, r.numel()), self.gen) for r in self._module_rows(S, W, obs.device)]
        acc: Dict[str, float] = {}
        kl_sum = [0.0] * len(streams)
        n = 0
        while min(st.covered for st in streams) < max(1, int(cfg.num_epochs)):
            total = None
            mstats: Dict[str, torch.Tensor] = {}
            for j, (pol, st) in enumerate(zip(m.policies, streams)):
                idx = st.next()
                b = {k: v[idx] for k, v in flat.items()}
                mean, log_std, values = self._forward(pol, obs, idx)
                loss, sts = ppo_loss(cfg, mean, log_std, values, b, self.kl_coeffs[j])
                total = loss if total is None else total + loss
                if "mean_kl" in sts:
                    kl_sum[j] += float(sts["mean_kl"].detach())
                for k, v in sts.items():
                    mstats[k] = mstats.get(k, 0.0) + v.detach() / len(streams)
            self.opt.zero_grad(set_to_none=True)
            total.backward()
            allreduce_grads([p for p in m.parameters() if p.grad is not None])
            if cfg.grad_clip:
                for pol in m.policies:  # each module's gradients by its own global norm
                    ps = [p for p in pol.parameters() if p.grad is not None]
                    if ps:
                        torch.nn.utils.clip_grad_norm_(ps, cfg.grad_clip)
            self.opt.step()
            for k, v in mstats.items():
                acc[k] = acc.get(k, 0.0) + float(v)
            n += 1
        out = {k: v / max(n, 1) for k, v in acc.items()}
        out["num_minibatch_steps"] = n
        if cfg.use_kl_loss:  # RLlib's adaptive KL coefficient, per module
            if self.world > 1:  # the ranks' mean KL: every rank keeps the same coefficients
                t = torch.tensor(kl_sum, dtype=torch.float64, device=obs.device)
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                kl_sum = [float(x) / self.world for x in t.tolist()]
            for j in range(len(streams)):
                kl = kl_sum[j] / max(n, 1)
                if kl > 2.0 * cfg.kl_target:
                    self.kl_coeffs[j] *= 1.5
                elif kl < 0.5 * cfg.kl_target:
                    self.kl_coeffs[j] *= 0.5
            out["kl_coeff"] = float(np.mean(self.kl_coeffs))
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
    env = VecInventoryEnv(None, 1, spec=spec, device=device, env_seeds=np.array([env_seed], dtype=np.uint32),
                          episode_ahead=0)
    rng = np.random.default_rng(action_seed)
    W, K, T, L = spec.W, spec.K, spec.episode_length, spec.n_features
    # samples stay on the device, [episode][step 0..T][agent][L] (agent order, the terminal observation
    # of each episode last), and come to the host once; no host round trip per step
    samples = torch.empty((n_episodes, T + 1, W, L), dtype=torch.float32, device=env.device)
    obs = env.reset()
    for ep in range(n_episodes):
        # one episode's actions in one draw: rng.uniform(size=(T, W, K)) is the same stream as the
        # reference's per-step, per-agent uniform(size=(K,)) calls, in the same order
        acts = torch.from_numpy(rng.uniform(-1, 1, size=(T, W, K)).astype(np.float32)).to(env.device)
        for t in range(T):
            samples[ep, t].copy_(obs[0])
            obs, _, trunc, final = env.step(acts[t].unsqueeze(0))
        samples[ep, T].copy_(final[0])
    all_obs = samples.reshape(-1, L).cpu().numpy()  # [(T + 1) * n_episodes * W, L]
    env.close()
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
        # weak partition: rank g steps global env ids [g E, (g + 1) E); ranks sharing a device split
        # the episode-ahead memory budget
        self.env = VecInventoryEnv(None, E, spec=self.spec, device=device, base_seed=self.train_seed,
                                   env_index_offset=mdist.shard(E, "weak", self.rank, self.world)[1],
                                   ea_mem_fraction=mdist.ea_mem_fraction())
        rc = cfg.rollout_config()
        torch.manual_seed(self.train_seed)
        W, L = self.env.W, self.env.local_obs_dim
        self.module = MultiAgentActorCritic(W, L, L * W, self.env.K, rc, cfg.parameter_sharing).to(self.device)
        if self.world > 1:  # identical initial weights on every rank
            for p in self.module.parameters():
                dist.broadcast(p.data, src=0)
        self.learner = PPOLearner(self.module, cfg, seed=self.train_seed + self.rank)
        # advantages standardised per module (RLlib's GAE connector): one group for the shared policy,
        # one per agent otherwise
        # one noise seed for every rank: the noise is keyed by global env id (msc_normal_keyed)
        self.collector = RolloutCollector(self.env, self.module, self.T, seed=self.train_seed + 1000,
                                          adv_groups=1 if cfg.parameter_sharing else W,
                                          obs_filter="meanstd" if cfg.obs_normalization == "meanstd" else "off")
        self.env.reset()
        self.iteration = 0
        self.timesteps = 0
        self._ep_ret = torch.zeros(E, dtype=torch.float64, device=self.device)
        # RLlib's metrics_num_episodes_for_smoothing = num_eval_episodes (mappo.py:177): the train
        # return is the mean of the last num_eval_episodes completed episodes
        self._completed: deque = deque(maxlen=max(1, int(cfg.num_eval_episodes)))
        self._n_episodes = 0

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
                ended = self._ep_ret[trunc[t]].tolist()
                self._completed.extend(ended)
                self._n_episodes += len(ended)
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
        ret_mean, n_ep = self._global_train_return()
        res = {"training_iteration": self.iteration, "num_env_steps_sampled_lifetime": self.timesteps,
               "train/episode_return_mean": ret_mean, "train/episodes": n_ep}
        res.update({f"learner/{k}": v for k, v in stats.items()})
        return res

    def _global_train_return(self):
        """(mean return of the smoothing windows of every rank, episodes completed on every rank).
        RLlib aggregates episode metrics over all env runners; here every rank contributes its window
        (sum, count) to one SUM all-reduce, so every rank reports -- and bases checkpoint_best on --
        the same value (marlsc/experiment.py)."""
        done = list(self._completed)
        if self.world == 1:
            return (float(np.mean(done)) if done else None), self._n_episodes
        t = torch.tensor([float(np.sum(done)) if done else 0.0, float(len(done)), float(self._n_episodes)],
                         dtype=torch.float64, device=self._ep_ret.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        s, c, n = t.tolist()
        return (s / c if c > 0 else None), int(n)

    @torch.no_grad()
    def evaluate(self, n_episodes: Optional[int] = None, seed: Optional[int] = None) -> Dict[str, Any]:
        """Deterministic (mean-action) evaluation episodes ('val' data mode).

        The reference evaluates on ONE env built with seed=eval_seed (no per-env seed derivation in
        'val' mode, src/algorithms/base.py:405-417) and num_eval_episodes set, running its episodes
        one after another; reset k derives the episode root SeedSequence([eval_seed, k]) and the
        counter cycles back to 0 after num_eval_episodes (multi_env.py:220-224). Here the n
        episodes run side by side: n envs with root eval_seed whose episode counters start at
        0..n-1, so env k plays exactly the reference's eval episode k."""
        from .spec import EnvSpec
        from .vec_env import VecInventoryEnv
        n = int(n_episodes or self.cfg.num_eval_episodes)
        meta = dict(self.env_meta)
        meta["data_mode"] = "val"
        meta["num_eval_episodes"] = n
        spec = EnvSpec.from_config(self.env_config, meta)
        root = self.eval_seed if seed is None else int(seed)
        env = VecInventoryEnv(None, n, spec=spec, device=self.device.index,
                              env_seeds=np.full(n, root & 0xFFFFFFFF, dtype=np.uint32), episode_ahead=0)
        env.set_episode_counters(np.arange(n, dtype=np.int32))
        obs = env.reset()
        full_fn = self._full_fn()
        filt = self.collector.obs_filter  # "meanstd": the trained filter with update=False
        ret = torch.zeros(n, dtype=torch.float64, device=self.device)
        for _ in range(spec.episode_length):
            if filt is not None:
                obs = filt.normalize(obs)
            full = env.obs_flat(obs=obs) if full_fn is not None else None
            mean, _ = self.module.dist_inputs(obs, full)
            obs, rew, trunc, _ = env.step(mean.clamp(-1.0, 1.0).contiguous())
            ret += rew.double().sum(-1)
        env.close()
        r = ret.cpu().numpy()
        return {"eval/episode_return_mean": float(r.mean()), "eval/episode_return_std": float(r.std()),
                "eval/episodes": n}

    # -- checkpoints ------------------------------------------------------------------------------
    # learner_state.pt (rank 0): module, optimizer, KL coefficients, counters; state.json: configs and
    # observation statistics; runtime_rank<r>.pt (every rank): the rank's env state blob
    # (msc_env_save_state, pending pre-generated demand included), its current observations, the
    # rollout / learner generators and the running episode returns -- so a resumed run continues
    # exactly where the saved one stopped instead of replaying its first iteration.
    def save_checkpoint(self, path: Union[str, Path]) -> Path:
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        if self.rank == 0:
            filt = self.collector.obs_filter
            torch.save({"module": self.module.state_dict(), "optimizer": self.learner.opt.state_dict(),
                        "kl_coeffs": list(self.learner.kl_coeffs), "iteration": self.iteration,
                        "timesteps": self.timesteps,
                        "obs_filter": None if filt is None else filt.state_dict()}, p / "learner_state.pt")
            stats = self.env_meta.get("obs_stats")
            (p / "state.json").write_text(json.dumps({
                "iteration": self.iteration, "timesteps": self.timesteps, "root_seed": self.root_seed,
                "world_size": self.world, "algorithm": asdict(self.cfg),
                "obs_stats": None if stats is None else [np.asarray(stats[0]).tolist(), np.asarray(stats[1]).tolist()]},
                indent=1))
        blob = self.env.save_state()
        torch.save({"env_state": torch.frombuffer(bytearray(blob), dtype=torch.uint8),
                    "obs": self.env.obs.detach().cpu(), "t_sync": int(getattr(self.env, "_t_sync", -1)),
                    "noise_step": int(self.collector.noise_step), "learner_gen": self.learner.gen.get_state(),
                    "ep_ret": self._ep_ret.detach().cpu(), "completed": list(self._completed),
                    "n_episodes": self._n_episodes,
                    "obs_filtered": [bool(ln.obs_filtered) for ln in self.collector._lanes]},
                   p / f"runtime_rank{self.rank}.pt")
        return p

    def export_module_weights(self, path: Union[str, Path]) -> Path:
        """module_weights.pt: the state dict of the policy module agent 0 maps to (the shared policy,
        or agent 0's own), keys actor.* / critic.* / log_std as the reference RLModule's
        (src/utils/weight_transfer.py:15-33, runner.py:379-395)."""
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        torch.save(self.module.policies[0].state_dict(), p)
        return p

    def load_checkpoint(self, path: Union[str, Path], runtime: bool = True) -> None:
        """Restore the learner (and with runtime=True this rank's env / generator state: resume).
        A runtime resume needs the saved world size: each rank's env shard and sampled timesteps
        assume it."""
        p = Path(path)
        sj = p / "state.json"
        if runtime and sj.exists():
            saved_world = json.loads(sj.read_text()).get("world_size", self.world)
            if int(saved_world) != self.world:
                raise ValueError(f"{p} was saved by {saved_world} ranks, this run has {self.world}: resume with the "
                                 f"same rank count, or load the weights only (runtime=False)")
        st = torch.load(p / "learner_state.pt", map_location=self.device, weights_only=True)
        self.module.load_state_dict(st["module"])
        self.learner.opt.load_state_dict(st["optimizer"])
        if "kl_coeffs" in st:
            self.learner.kl_coeffs = [float(x) for x in st["kl_coeffs"]]
        else:  # round-1 checkpoints
            self.learner.kl_coeffs = [float(st["kl_coeff"])] * len(self.module.policies)
        self.iteration = int(st["iteration"])
        self.timesteps = int(st["timesteps"])
        if self.collector.obs_filter is not None:
            if st.get("obs_filter") is None:
                raise ValueError(f"{p}: obs_normalization 'meanstd' but the checkpoint holds no filter state")
            self.collector.obs_filter.load_state_dict(st["obs_filter"])
        rt_path = p / f"runtime_rank{self.rank}.pt"
        if not runtime or not rt_path.exists():  # module-only checkpoint: weights restored, sampling restarts
            return
        rt = torch.load(rt_path, map_location="cpu", weights_only=True)
        self.env.load_state(bytes(rt["env_state"].numpy().tobytes()))
        self.env.obs.copy_(rt["obs"].to(self.device))
        self.env._t_sync = int(rt["t_sync"])
        if "noise_step" in rt:
            self.collector.noise_step = int(rt["noise_step"])
        else:
            # round <= 3 checkpoints held a per-rank torch generator instead: every collect draws T
            # rollout steps of keyed noise, so the stream position is iterations x T (the resumed run
            # continues the keyed stream instead of replaying the steps already taken)
            self.collector.noise_step = self.iteration * self.collector.T
            warnings.warn(f"{p}: checkpoint without 'noise_step' (round <= 3); keyed action noise resumes at "
                          f"step {self.collector.noise_step} = iteration x T")
        self.learner.gen.set_state(rt["learner_gen"])
        self._ep_ret.copy_(rt["ep_ret"].to(self.device))
        self._completed = deque((float(x) for x in rt["completed"]), maxlen=self._completed.maxlen)
        self._n_episodes = int(rt["n_episodes"])
        for ln, f in zip(self.collector._lanes, rt.get("obs_filtered", [])):
            ln.obs_filtered = bool(f)
