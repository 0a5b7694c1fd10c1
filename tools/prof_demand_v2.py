"""Demand kernel alone (no pipelining, no step kernels beside it) at the C3 shape: the unit parser
against the f32-ring parser (MSC_DEMAND_IMPL=v2), HIP-event time per generate_demand; with
MSC_LIB_VARIANT=v2prof (make variant1 NAME=v2prof VFLAGS=-DMSC_PROF TU=demand_v2) also the f32
parser's in-kernel counters: rounds per wave and exact recomputations per launch."""
import ctypes as C
import os
import sys
from pathlib import Path

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
L = abi.lib()
prof = hasattr(L, "msc_debug_prof_v2")
buf = (C.c_ulonglong * 8)()
for impl in os.environ.get("IMPLS", "unit v2").split():
    os.environ["MSC_DEMAND_IMPL"] = impl
    env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=default_train_seed(42))
    env.set_pipelining(False)
    env.reset()
    act = torch.rand((E, 8, 5), device="cuda") * 2 - 1
    env.step(act)
    torch.cuda.synchronize()
    if prof:
        L.msc_debug_prof_v2(buf, 1)
    t = []
    for i in range(N):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.generate_demand()
        b.record()
        env.step(act)
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b))
    msg = f"impl={impl} quota={os.environ.get('MSC_V2_QUOTA', '-')} envs={E}: demand kernel alone {sum(t) / N:.4f} ms"
    if prof and impl == "v2":
        L.msc_debug_prof_v2(buf, 0)
        v = list(buf)
        waves = max(v[2], 1)
        msg += f"; rounds/wave {v[0] / waves:.0f}, exact recomputations per launch {v[1] / N:.1f}"
    print(msg, flush=True)
    env.close()
