"""Host enqueue cost of one env step at the C2 shape (8 x 64 x 5, 4,096 envs, episode-ahead demand):
bursts of steps enqueued right after a synchronize (the device queue never fills within a burst), timed
on the host, through VecInventoryEnv.step and through a bare ctypes call of msc_env_step with prebuilt
arguments; prints microseconds per step for each. Under `rocprofv3 --hip-runtime-trace --stats` the
same run gives the per-API split. Usage: python tools/host_overhead.py [bursts] [burst_len]"""
import ctypes as C
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
import torch  # noqa: E402

from marlsc import abi, make_synthetic_env_config  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

bursts = int(sys.argv[1]) if len(sys.argv) > 1 else 40
blen = int(sys.argv[2]) if len(sys.argv) > 2 else 25
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
E = 4096
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=7)
g = torch.Generator(device="cuda").manual_seed(1)
pool = [torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
env.reset()
for i in range(3000):  # episode-ahead demand into steady state
    env.step(pool[i % 8])
torch.cuda.synchronize()


def run(step):
    tot, n = 0.0, 0
    for _ in range(bursts):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(blen):
            step(i)
        tot += time.perf_counter() - t0
        n += blen
    torch.cuda.synchronize()
    return tot / n * 1e6


lib = abi.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
args = [(ptr(a), ptr(env.obs), ptr(env.rewards), None, ptr(env.truncated), ptr(env.final_obs), None, st)
        for a in pool]
h = env._h


def bare(i):
    rc = lib.msc_env_step(h, *args[i % 8])
    if rc:
        raise RuntimeError(abi.last_error() if hasattr(abi, "last_error") else rc)


def wrapped(i):
    env.step(pool[i % 8])


for name, f in (("VecInventoryEnv.step", wrapped), ("ctypes msc_env_step", bare), ("VecInventoryEnv.step (again)", wrapped)):
    print(f"{name:30s} {run(f):8.1f} us/step host", flush=True)
env.check()
