"""C2 IPPO rollout times rollout by rollout after a given number of env-only steps (the bench's c2
line warm-up + window + timing pass): shows whether the rollout rate depends on the episode-ahead
refill phase it starts in. Usage: PRE=<env steps> python tools/c2_rollout_phases.py"""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
sys.path.insert(0, str(REPO))
import torch  # noqa: E402
import yaml  # noqa: E402

import bench  # noqa: E402
from marlsc import make_synthetic_env_config  # noqa: E402
from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig  # noqa: E402
from marlsc.seeding import default_train_seed  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

algo = yaml.safe_load(open(REPO / "config_files/algorithms/ippo.yaml"))
cfg = make_synthetic_env_config(8, 64, 5)
meta = {"include_warehouse_id": True, "obs_normalization": "meanstd_custom"}
meta["obs_stats"] = bench.bench_obs_stats(cfg, meta)
spec = EnvSpec.from_config(cfg, meta)
E = 4096
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=default_train_seed(42))
g = torch.Generator(device="cuda").manual_seed(99)
pool = [torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
env.reset()
pre = int(os.environ.get("PRE", "4850"))
for i in range(pre):
    env.step(pool[i % 8])
torch.cuda.synchronize()
rc = RolloutConfig.from_algorithm_config(algo)
torch.manual_seed(0)
m = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
col = RolloutCollector(env, m, 100, seed=0)
out = []
for r in range(16):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    col.collect()
    torch.cuda.synchronize()
    out.append((time.perf_counter() - t0) / 100 * 1e3)
print(f"PRE={pre}: ms/step per rollout:", " ".join(f"{x:.3f}" for x in out))
