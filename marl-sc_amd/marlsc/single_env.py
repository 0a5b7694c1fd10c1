"""Single-agent (centralised, CPPO baseline) views of the env -- the reference's
`CentralizedEnvWrapper` (src/environment/envs/single_env.py:25-267) over this build's envs.

* `CentralizedEnvWrapper(env_config, seed, env_meta)`: the reference's gymnasium-style API over one
  `marlsc.InventoryEnvironment`: observation = the global vector concat(local_0 .. local_{W-1})
  (the tail of any agent's local || global observation, single_env.py:228-246), action = the flat
  (W*K,) vector split per warehouse in agent order (single_env.py:248-267), reward = the sum of
  the per-warehouse rewards in agent order, terminated / truncated = all agents'.
* `VecCentralizedEnv`: the same view over E envs of a `VecInventoryEnv` on the GPU:
  obs [E, W*L] (a view of the local observations, no copy), actions [E, W*K], rewards [E] f64
  (the agent-order sum of the f64 per-agent rewards), truncated [E].
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .env import Box, InventoryEnvironment
from .vec_env import VecInventoryEnv


class CentralizedEnvWrapper:
    metadata = {"render_modes": ["human"], "name": "single_env"}

    def __init__(self, env_config: Any, seed: Optional[int] = None, env_meta: Optional[Dict[str, Any]] = None,
                 device: int = 0):
        self.env = InventoryEnvironment(env_config, seed=seed, env_meta=env_meta, device=device)
        self.env_config = env_config
        self.n_warehouses = self.env.n_warehouses
        self.n_skus = self.env.n_skus
        self._local_obs_dim = self.env._compute_local_obs_dim()
        self._global_obs_dim = self.n_warehouses * self._local_obs_dim
        self.observation_space = Box(-np.inf, np.inf, (self._global_obs_dim,), np.float32)
        self.action_space = Box(-1.0, 1.0, (self.n_warehouses * self.n_skus,), np.float32)

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        obs, infos = self.env.reset(seed=seed, options=options)
        return self._extract_global_obs(obs), infos.get(self.env.agents[0], {})

    def step(self, action: np.ndarray) -> Tuple[np.ndarray, float, bool, bool, Dict[str, Any]]:
        obs, rewards, terms, truncs, infos = self.env.step(self._split_action(action))
        total = 0.0
        for a in self.env.agents:  # sum(rewards.values()) in agent order
            total += rewards[a]
        return (self._extract_global_obs(obs), total, all(terms.values()), all(truncs.values()),
                infos.get(self.env.agents[0], {}))

    def render(self):
        self.env.render()

    def close(self):
        self.env.close()

    # forwarded properties (single_env.py:160-224)
    @property
    def collect_step_info(self) -> bool:
        return self.env.collect_step_info

    @collect_step_info.setter
    def collect_step_info(self, value: bool):
        self.env.collect_step_info = value

    @property
    def agents(self):
        return self.env.agents

    @property
    def episode_length(self) -> int:
        return self.env.episode_length

    @property
    def max_expected_lead_time(self) -> int:
        return self.env.max_expected_lead_time

    @property
    def feature_config(self):
        return self.env.feature_config

    @property
    def include_warehouse_id(self) -> bool:
        return self.env.include_warehouse_id

    @property
    def rolling_window(self) -> int:
        return self.env.rolling_window

    @property
    def obs_normalization(self):
        return self.env.obs_normalization

    @property
    def obs_stats(self):
        return self.env.obs_stats

    def _extract_global_obs(self, obs_dict: Dict[str, np.ndarray]) -> np.ndarray:
        return obs_dict[self.env.agents[0]][self._local_obs_dim:]

    def _split_action(self, action: np.ndarray) -> Dict[str, np.ndarray]:
        K = self.n_skus
        action = np.asarray(action)
        return {a: action[i * K:(i + 1) * K] for i, a in enumerate(self.env.agents)}


class VecCentralizedEnv:
    """E centralised envs in lockstep on one GPU (torch device tensors in and out)."""

    def __init__(self, env: VecInventoryEnv):
        self.venv = env
        self.n_envs, self.W, self.K, self.L = env.n_envs, env.W, env.K, env.local_obs_dim
        self.observation_space = Box(-np.inf, np.inf, (self.W * self.L,), np.float32)
        self.action_space = Box(-1.0, 1.0, (self.W * self.K,), np.float32)

    def _glob(self, obs: torch.Tensor) -> torch.Tensor:
        return obs.view(self.n_envs, self.W * self.L)  # concat(local_0 .. local_{W-1}) per env

    def reset(self, **kw) -> torch.Tensor:
        return self._glob(self.venv.reset(**kw))

    def step(self, actions: torch.Tensor):
        a = actions.reshape(self.n_envs, self.W, self.K)
        obs, _, trunc, final = self.venv.step(a.contiguous(), want_f64=True)
        r = self.venv.rewards_f64
        total = r[:, 0].clone()
        for w in range(1, self.W):  # agent-order sum of the f64 per-agent rewards
            total += r[:, w]
        return self._glob(obs), total, trunc, (None if final is None else self._glob(final))
