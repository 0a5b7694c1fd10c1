"""Host-side cost of one rollout collect (C2 IPPO / C3 MAPPO shapes): wall time with a device sync,
the time until collect() returns (host enqueue), and a cProfile of the enqueue path.
Usage: python tools/prof_rollout_host.py [c2|c3]"""
import cProfile
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "marl-sc_amd"), str(REPO)]

import torch  # noqa: E402
import yaml  # noqa: E402

from marlsc import make_synthetic_env_config  # noqa: E402
from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig  # noqa: E402
from marlsc.seeding import default_train_seed  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c2"
E, algo_name = (4096, "ippo") if which == "c2" else (32768, "mappo")
algo = yaml.safe_load(open(REPO / f"config_files/algorithms/{algo_name}.yaml"))
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=default_train_seed(42))
env.reset()
rc = RolloutConfig.from_algorithm_config(algo)
torch.manual_seed(0)
m = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
col = RolloutCollector(env, m, spec.episode_length, seed=0)
for _ in range(3):
    col.collect()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    col.collect()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{which}: collect of {spec.episode_length} steps: host enqueue {1e3 * (t1 - t0) / spec.episode_length:.4f} ms/step, "
          f"wall {1e3 * (t2 - t0) / spec.episode_length:.4f} ms/step", flush=True)
pr = cProfile.Profile()
pr.enable()
col.collect()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
