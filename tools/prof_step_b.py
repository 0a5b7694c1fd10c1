"""In-kernel cycle accounting of the group allocator (step_b_kernel) at the C5 shape (profiling build,
`make -C marl-sc_amd prof`): 16 warehouses x 256 regions x 5 SKUs, 8,192 envs, empirical demand from a
synthetic trace (as bench.py --config c5). Prints per-wave cycles of the order loop, the region
epilogues, the allocation rounds, and the per-order remainder (record window + bookkeeping).
Usage: python tools/prof_step_b.py [envs] [steps]"""
import ctypes as C
import os
import sys
from pathlib import Path

os.environ["MSC_LIB_VARIANT"] = "prof"
os.environ.setdefault("MSC_ALLOC_IMPL", "group")
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
import torch  # noqa: E402

from marlsc import abi  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
from marlsc import make_synthetic_env_config  # noqa: E402
from marlsc.synthetic import make_synthetic_trace  # noqa: E402

cfg = make_synthetic_env_config(16, 256, 5)  # as bench.py c5_line
cfg["components"]["demand_sampler"] = {"type": "empirical", "params": None}
meta = {"include_warehouse_id": True, "demand_trace": make_synthetic_trace(256, 5, 300, orders_per_step=(200, 1000), seed=0)}
spec = EnvSpec.from_config(cfg, meta)
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=11)
env.reset()
g = torch.Generator(device="cuda").manual_seed(3)
act = torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1
L = abi.lib()
buf = (C.c_ulonglong * 16)()
for _ in range(5):
    env.step(act)
torch.cuda.synchronize()
L.msc_debug_prof(buf, 1)
t = []
for i in range(N):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    env.step(act)
    b.record()
    torch.cuda.synchronize()
    t.append(a.elapsed_time(b))
L.msc_debug_prof(buf, 0)
v = list(buf)
sw = max(v[15] / N, 1)  # step_b waves per launch
per = lambda i: v[i] / N / sw  # noqa: E731
print(f"step (all kernels) {sum(t) / N:.3f} ms avg over {N}; step_b waves/launch {sw:.0f}")
print(f"step_b cycles/wave: order loop {per(10):.0f}  region changes (any env of the wave) {per(11):.0f}  allocation rounds {per(12):.0f}  "
      f"rest (records, bookkeeping) {per(10) - per(11) - per(12):.0f}")
print(f"allocation iterations/wave (lane 0) {per(13):.0f}  region-change passes/wave {per(14):.0f}")
env.check()
