"""In-kernel cycle accounting of the demand kernel (profiling build, `make -C marl-sc_amd prof`).

Runs the bench workload's demand generation N times through libmarlsc_prof.so and prints the
per-wave averages of the MSC_PROF counters (cycles in settle passes / barriers, hot rounds, ...).
"""
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
L.msc_debug_prof(buf, 0)
v = list(buf)
waves = v[6] / N
per = lambda i: v[i] / N / max(waves, 1)  # noqa: E731
print(f"demand kernel {sum(t)/N:.3f} ms avg; parser waves/launch {waves:.0f}")
print(f"parser cycles/wave: total {per(0):.0f}  settle {per(1):.0f}  barrier {per(2):.0f}  "
      f"hot+other {per(0)-per(1)-per(2):.0f}")
print(f"settles/wave {per(3):.0f}  rounds/wave {per(4):.0f}  chunks/wave {per(5):.0f}")
print(f"cycles per settle {v[1]/max(v[3],1):.0f}; per round (excl settles) {(v[0]-v[1]-v[2])/max(v[4],1):.0f}")
gw = max(waves, 1) * int(os.environ.get("GEN", "2"))
print(f"generator cycles/wave: gen {v[8]/N/gw:.0f}  barrier {v[9]/N/gw:.0f}")
sw = max(v[15] / N, 1)
print(f"step_b cycles/wave: order loop {v[10]/N/sw:.0f}  region epilogues {v[11]/N/sw:.0f}  allocation {v[12]/N/sw:.0f}  "
      f"allocation iterations (lane 0) {v[13]/N/sw:.0f}  epilogue passes {v[14]/N/sw:.0f}")
