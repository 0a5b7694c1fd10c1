"""In-kernel cycle accounting of the split-parser demand kernel (profiling build, `make -C marl-sc_amd
prof`): per-wave averages of the chain parser A, the bookkeeper B and the generator waves (cycles,
cycles at chunk barriers, B's replay cycles, A's rounds), plus the old unit parser's counters for
comparison. Runs the bench workload's demand generation alone (no pipelining)."""
import ctypes as C
import os
import sys
from pathlib import Path

os.environ["MSC_LIB_VARIANT"] = "prof"
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
import torch  # noqa: E402

from marlsc import abi, make_synthetic_env_config  # noqa: E402
from marlsc.seeding import default_train_seed  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

E = int(os.environ.get("ENVS", "32768"))
N = int(os.environ.get("REPS", "20"))
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=default_train_seed(42))
env.set_pipelining(False)
env.reset()
act = torch.rand((E, 8, 5), device="cuda") * 2 - 1
L = abi.lib()
buf = (C.c_ulonglong * 16)()
env.step(act)
torch.cuda.synchronize()
L.msc_debug_prof_ab(buf, 1)
L.msc_debug_prof(buf, 1)
t = []
for i in range(N):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    env.generate_demand()
    b.record()
    env.step(act)
    torch.cuda.synchronize()
    t.append(a.elapsed_time(b))
print(f"impl={os.environ.get('MSC_DEMAND_IMPL', 'default')} envs={E}: demand kernel {sum(t) / N:.3f} ms avg")
L.msc_debug_prof_ab(buf, 0)
v = list(buf)
if v[3]:
    aw, gw = v[3] / N, max(v[9] / N, 1)
    print(f"A (chain parser): {aw:.0f} waves/launch, cycles/wave {v[0] / N / aw:.0f}, at barriers {v[1] / N / aw:.0f}, "
          f"rounds {v[2] / N / aw:.0f}, cycles per round outside barriers {(v[0] - v[1]) / max(v[2], 1):.0f}")
    print(f"B (bookkeeper): cycles/wave {v[4] / N / aw:.0f}, at barriers {v[5] / N / aw:.0f}, replaying {v[6] / N / aw:.0f}")
    print(f"generators: {gw:.0f} waves/launch, cycles/wave {v[7] / N / gw:.0f}, at barriers {v[8] / N / gw:.0f}")
L.msc_debug_prof(buf, 0)
v = list(buf)
if v[6]:
    waves = v[6] / N
    print(f"unit parser: cycles/wave {v[0] / N / waves:.0f}, barrier {v[2] / N / waves:.0f}, rounds/wave {v[4] / N / waves:.0f}")
