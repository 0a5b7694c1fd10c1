"""Host-side SeedManager with the reference's seed semantics (src/utils/seed_manager.py).

Experiment-level seeds (train / eval / obs_stats ...) are derived on the host with numpy's
SeedSequence exactly as the reference does; the per-env, per-episode seeding of the
environment components happens on the device (csrc/rng.hpp, reset kernel).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
from numpy.random import SeedSequence

EXPERIMENT_SEEDS: Tuple[str, ...] = ("data_weights", "data_distances", "data_costs", "train", "eval", "obs_stats")
ENVIRONMENT_SEEDS: Tuple[str, ...] = ("preprocessing", "inventory", "demand_sampler", "lead_time_sampler")
STOCHASTIC_SEEDS: Tuple[str, ...] = ("demand_sampler", "lead_time_sampler")


class SeedManager:
    """Same contract as the reference class (seed_manager.py:34-224)."""

    def __init__(self, root_seed: Optional[int] = None, seed_registry: Tuple[str, ...] = EXPERIMENT_SEEDS):
        self.root_seed = root_seed
        self._original_root_seed = root_seed
        self._episode_counter = 0
        self._seed_registry = seed_registry
        self._seed_sequences: Dict[str, Optional[SeedSequence]] = {}
        self._spawn_seeds()

    def get_rng(self, name: str) -> np.random.Generator:
        return np.random.default_rng(self._get_seed_sequence(name))

    def get_seed_int(self, name: str) -> Optional[int]:
        ss = self._get_seed_sequence(name)
        return None if ss is None else int(ss.generate_state(1, dtype=np.uint32)[0])

    def advance_episode(self) -> None:
        if self._original_root_seed is None:
            return
        self.root_seed = int(SeedSequence([self._original_root_seed, self._episode_counter])
                             .generate_state(1, dtype=np.uint32)[0])
        self._spawn_seeds()
        self._episode_counter += 1

    def update_root_seed(self, root_seed: Optional[int]) -> None:
        self.root_seed = root_seed
        self._original_root_seed = root_seed
        self._episode_counter = 0
        self._spawn_seeds()

    def spawn_child_seeds(self, name: str, n: int) -> List[Optional[int]]:
        ss = self._get_seed_sequence(name)
        if ss is None:
            return [None] * n
        return [int(c.generate_state(1, dtype=np.uint32)[0]) for c in ss.spawn(n)]

    @staticmethod
    def derive_env_seed(base_seed: int, worker_index: int, env_index: int) -> int:
        return int(SeedSequence([base_seed, worker_index, env_index]).generate_state(1, dtype=np.uint32)[0])

    def _get_seed_sequence(self, name: str) -> Optional[SeedSequence]:
        if name not in self._seed_registry:
            raise ValueError(f"Seed '{name}' not in registry {self._seed_registry}")
        return self._seed_sequences[name]

    def _spawn_seeds(self) -> None:
        if self.root_seed is None:
            self._seed_sequences = {n: None for n in self._seed_registry}
            return
        children = SeedSequence(self.root_seed).spawn(len(self._seed_registry))
        self._seed_sequences = dict(zip(self._seed_registry, children))


def default_train_seed(root_seed: int = 42) -> int:
    """train_seed of an experiment with root seed `root_seed` (runner.py:59-73)."""
    return SeedManager(root_seed).get_seed_int("train")
