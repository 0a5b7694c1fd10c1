"""PettingZoo-style drop-in for the reference's `InventoryEnvironment`
(src/environment/envs/multi_env.py:38-437): same constructor `(env_config, seed, env_meta)`,
same `reset()` / `step()` dict API, agent ids, spaces and attributes read by callers, backed by
a batch-of-one `VecInventoryEnv` on the GPU (the HIP kernels do all the work).

Observations per agent are the reference's flat vector `local || global`
(multi_env.py:548-575); rewards are Python floats from the f64 rewards; infos carry the
`collect_step_info` dict (multi_env.py:330-361) when `collect_step_info = True`.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import numpy as np
import torch

from .spec import EnvSpec
from .vec_env import VecInventoryEnv


class Box:
    """Minimal gymnasium.spaces.Box stand-in (gymnasium is not a dependency)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


class InventoryEnvironment:
    metadata = {"render_modes": ["human"], "name": "multi_env"}

    def __init__(self, env_config: Any, seed: Optional[int] = None, env_meta: Optional[Dict[str, Any]] = None,
                 *, device: int = 0):
        env_meta = dict(env_meta or {})
        self.env_config = env_config
        self.spec = EnvSpec.from_config(env_config, env_meta, allow_nr_ne_nw=True)
        self._seeded_at_construction = seed is not None
        root = int(seed) if seed is not None else int.from_bytes(os.urandom(4), "little")
        self._vec = VecInventoryEnv(None, 1, spec=self.spec, device=device, env_seeds=[root], episode_ahead=0)
        self.n_warehouses, self.n_skus, self.n_regions = self.spec.W, self.spec.K, self.spec.R
        self.episode_length = self.spec.episode_length
        self.feature_config = self.spec.features
        self.max_expected_lead_time = self.spec.max_expected_lead_time
        self.rolling_window = 5
        self.ema_alpha = 0.3
        self.obs_normalization = env_meta.get("obs_normalization", "off")
        self.obs_stats = env_meta.get("obs_stats")
        self.include_warehouse_id = bool(env_meta.get("include_warehouse_id", False))
        self._num_eval_episodes = env_meta.get("num_eval_episodes")
        self.agents = [f"warehouse_{i}" for i in range(self.n_warehouses)]
        self.possible_agents = list(self.agents)
        self.collect_step_info = False
        self.timestep = 0
        self._auto_reset_pending = False
        self._L = self.spec.local_obs_dim

    # -- reference helpers ----------------------------------------------------------------------
    def _compute_local_obs_dim(self) -> int:
        return self._L

    def observation_space(self, agent: str) -> Box:
        return Box(-np.inf, np.inf, (self._L * (1 + self.n_warehouses),), np.float32)

    def global_observation_space(self) -> Box:
        return Box(-np.inf, np.inf, (self._L * self.n_warehouses,), np.float32)

    def action_space(self, agent: str) -> Box:
        return Box(-1.0, 1.0, (self.n_skus,), np.float32)

    def render(self):
        pass

    @property
    def inventory(self) -> np.ndarray:
        return self._vec.read_state()["inventory"][0].astype(np.float64)

    def _obs_dict(self, local: torch.Tensor) -> Dict[str, np.ndarray]:
        loc = local[0].detach().cpu().numpy()
        glob = loc.reshape(-1)
        return {a: np.concatenate([loc[i], glob]) for i, a in enumerate(self.agents)}

    # -- API ----------------------------------------------------------------------------------
    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        """multi_env.py:192-251. If an auto-reset already happened at truncation, the fresh
        episode it started is returned (unless a seed forces re-seeding)."""
        if self._seeded_at_construction:
            restart = seed is not None and self._num_eval_episodes is not None
            if self._auto_reset_pending and not restart:
                obs = self._pending_obs
            else:
                obs = self._vec.reset(eval_restart=restart)
        elif seed is not None:
            obs = self._vec.reset(root_seeds=torch.tensor([int(seed) & 0xFFFFFFFF], device=self._vec.device))
        else:
            obs = self._pending_obs if self._auto_reset_pending else self._vec.reset()
        self._auto_reset_pending = False
        self.timestep = 0
        return self._obs_dict(obs), {a: {} for a in self.agents}

    def step(self, actions: Dict[str, np.ndarray]):
        """multi_env.py:253-366."""
        act = np.stack([np.asarray(actions[a], dtype=np.float32) for a in self.agents])[None]
        info = self._vec.alloc_info() if self.collect_step_info else None
        obs, rew, tr, fo = self._vec.step(torch.from_numpy(act).to(self._vec.device), want_f64=True, info=info)
        truncated = bool(tr[0].item())
        self.timestep += 1
        if truncated:
            self._pending_obs = obs.clone()
            self._auto_reset_pending = True
            obs_d = self._obs_dict(fo)
        else:
            obs_d = self._obs_dict(obs)
        r64 = self._vec.rewards_f64[0].cpu().numpy()
        rewards = {a: float(r64[i]) for i, a in enumerate(self.agents)}
        terms = {a: False for a in self.agents}
        truncs = {a: truncated for a in self.agents}
        if info is not None:
            h = {k: v[0].cpu().numpy() for k, v in info.items()}
            n_orders = int(h["n_orders"])
            step_info = {
                "inventory": h["inventory_before"].astype(np.float64),
                "pending_total": h["pending_total"].astype(np.float32),
                "order_quantities": h["order_quantities"].astype(np.float64),
                "demand_per_region": h["demand_per_region"].astype(np.float64),
                "fulfilled_per_warehouse": h["fulfilled_per_warehouse"].astype(np.float64),
                "unfulfilled_demands": h["unfulfilled_demands"].astype(np.float64),
                "shipment_counts": h["shipment_counts"].astype(np.int64),
                "shipment_quantities": h["shipment_quantities"].astype(np.float64),
                "shipment_quantities_by_sku": h["shipment_quantities_by_sku"].astype(np.float64),
                "lost_order_counts": h["lost_order_counts"].astype(np.int64),
                "lost_sales": h["lost_sales"],
                "n_orders": n_orders,
                "holding_cost": h["costs"][0], "penalty_cost": h["costs"][1],
                "outbound_shipment_cost": h["costs"][2], "inbound_shipment_cost": h["costs"][3],
            }
            infos = {a: step_info for a in self.agents}
        else:
            infos = {a: {} for a in self.agents}
        return obs_d, rewards, terms, truncs, infos

    def close(self):
        self._vec.close()
