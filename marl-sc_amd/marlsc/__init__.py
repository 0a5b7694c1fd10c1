"""marlsc -- MI355X-native vectorised multi-agent supply-chain environment + rollout.

Hot path (BASELINE.json north_star): the reference's `InventoryEnvironment.step()/reset()`
(src/environment/envs/multi_env.py:192-366) and its five components, as HIP kernels for gfx950
behind the C ABI in include/marlsc.h (libmarlsc.so); GAE as a HIP reverse-scan kernel.
Host modules here only parse configs, pack descriptors and pass torch device pointers.
"""
from .config import ConfigNode, load_environment_config, load_feature_config, validate_environment_config
from .seeding import SeedManager, default_train_seed
from .spec import EnvSpec
from .synthetic import make_synthetic_env_config

__all__ = [
    "ConfigNode", "load_environment_config", "load_feature_config", "validate_environment_config",
    "SeedManager", "default_train_seed", "EnvSpec", "make_synthetic_env_config",
    "VecInventoryEnv", "InventoryEnvironment", "CentralizedEnvWrapper", "VecCentralizedEnv",
]


def __getattr__(name):  # torch-dependent modules load lazily
    if name == "VecInventoryEnv":
        from .vec_env import VecInventoryEnv
        return VecInventoryEnv
    if name == "InventoryEnvironment":
        from .env import InventoryEnvironment
        return InventoryEnvironment
    if name in ("CentralizedEnvWrapper", "VecCentralizedEnv"):
        from . import single_env
        return getattr(single_env, name)
    raise AttributeError(name)
