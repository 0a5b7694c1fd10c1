"""In-kernel cycle accounting of the scan allocator (profiling build, `make -C marl-sc_amd prof`):
per-wave cycles of the whole order loop, of the window ranking and of the region epilogues, at
the configs[1] shape (4,096 envs, episode-ahead demand), averaged over REPS steps."""
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

E = int(os.environ.get("ENVS", "4096"))
N = int(os.environ.get("REPS", "50"))
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=default_train_seed(42))
env.reset()
act = torch.rand((E, 8, 5), device="cuda") * 2 - 1
L = abi.lib()
buf = (C.c_ulonglong * 8)()
for _ in range(int(os.environ.get("WARM", "250"))):
    env.step(act)
torch.cuda.synchronize()
L.msc_debug_prof_scan(buf, 1)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for i in range(N):
    env.step(act)
b.record()
torch.cuda.synchronize()
L.msc_debug_prof_scan(buf, 0)
v = list(buf)
w = max(v[5], 1)
print(f"{N} steps in {a.elapsed_time(b) / N:.3f} ms/step; waves {v[5] / N:.0f} per step")
print(f"per wave: cycles {v[0] / w:.0f}, ranking {v[1] / w:.0f}, epilogues {v[2] / w:.0f} ({v[3] / w:.1f} of them), "
      f"orders {v[4] / w:.1f}; chain cycles per order (excl. ranking, epilogues) "
      f"{(v[0] - v[1] - v[2]) / max(v[4], 1):.0f}; cycles per epilogue {v[2] / max(v[3], 1):.0f}; "
      f"batches {v[6] / w:.1f} ({v[4] / max(v[6], 1):.2f} orders each)")
if v[7]:
    print(f"shader clock while the loop ran: {v[0] / v[7] * 100:.0f} MHz (clock64 cycles / 100 MHz wall-clock ticks), "
          f"loop wall {v[7] / w / 100:.1f} us per wave")
