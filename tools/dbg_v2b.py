import os, sys
sys.path.insert(0, "marl-sc_amd")
import numpy as np, torch
from marlsc import make_synthetic_env_config
from marlsc.spec import EnvSpec
from marlsc.vec_env import VecInventoryEnv
cfg = make_synthetic_env_config(5, 24, 5, episode_length=7, probability_skus=0.3)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
res = {}
for impl in ("unit", "v2"):
    os.environ["MSC_DEMAND_IMPL"] = impl
    os.environ["MSC_EA"] = "0"
    env = VecInventoryEnv(None, 64, spec=spec, device=0, base_seed=777)
    env.set_pipelining(False)
    env.reset()
    a = torch.zeros((64, 5, 5), device="cuda")
    info = env.alloc_info()
    env.step(a, info=info)
    res[impl] = {k: v.detach().cpu().numpy().copy() for k, v in info.items()}
    print(impl, env.kernel_choice(), list(info.keys()))
    env.close()
d = res["unit"]["demand_per_region"] if "demand_per_region" in res["unit"] else None
for k in res["unit"]:
    if not np.array_equal(res["unit"][k], res["v2"][k]):
        u, v = res["unit"][k], res["v2"][k]
        bad = np.argwhere(u != v)
        print("DIFF", k, u.shape, "first", bad[:3].tolist())
        e = bad[0][0]
        print(" unit", u[e].tolist()[:8])
        print(" v2  ", v[e].tolist()[:8])
