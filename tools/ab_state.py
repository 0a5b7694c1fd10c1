"""Which earlier action in a process slows the C2 env step (bench.py's c2 line runs after the
headline, the rollout and two timed micro-benchmarks): time 1,000 C2 steps, then after each
candidate action again, in one process."""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
import torch  # noqa: E402

from marlsc import make_synthetic_env_config  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402
from marlsc.vec_env import VecInventoryEnv  # noqa: E402

E = int(os.environ.get("ENVS", "4096"))
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=1234)
acts = [torch.rand((E, 8, 5), device="cuda") * 2 - 1 for _ in range(8)]
env.reset()
for i in range(1000):
    env.step(acts[i % 8])
torch.cuda.synchronize()


def timed(tag, n=1000):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        env.step(acts[i % 8])
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{tag:28s} {dt / n * 1e3:.4f} ms/step  host {th / n * 1e3:.4f} ms/step  {E * 8 * n / dt / 1e6:.1f} M", flush=True)


timed("baseline")
timed("baseline again")
# timing-enabled torch events on the default stream
ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ea.record()
x = torch.randn(1 << 20, device="cuda")
eb.record()
torch.cuda.synchronize()
_ = ea.elapsed_time(eb)
timed("after timing events")
# the fused MLP micro-benchmark
from marlsc.mlp import mlp3_forward  # noqa: E402
from marlsc.rollout import MLP  # noqa: E402
m = MLP(34, 5, {"hidden_sizes": [256, 256]}).cuda()
xg = torch.randn((262144, 34), device="cuda")
yo = torch.empty((262144, 5), device="cuda")
with torch.no_grad():
    for _ in range(5):
        mlp3_forward(list(m), xg, out=yo)
torch.cuda.synchronize()
timed("after mlp3 kernel")
# a large GAE
from marlsc.rollout import gae  # noqa: E402
T, N = 100, 262144
r_ = torch.randn((T, N), device="cuda")
v_ = torch.randn((T + 1, N), device="cuda")
nv_ = torch.randn((T, N), device="cuda")
te_ = torch.zeros((T, N), dtype=torch.uint8, device="cuda")
tr_ = torch.zeros((T, N), dtype=torch.uint8, device="cuda")
adv_, tgt_ = torch.empty_like(r_), torch.empty_like(r_)
st_ = torch.zeros((1, 3), dtype=torch.float64, device="cuda")
for _ in range(5):
    gae(r_, v_, nv_, te_, tr_, 0.99, 0.95, adv_, tgt_, st_)
torch.cuda.synchronize()
timed("after gae T=100")
del r_, v_, nv_, te_, tr_, adv_, tgt_
timed("after freeing gae buffers")
big = torch.empty(int(float(os.environ.get("BIG_GB", "8")) * (1 << 30)), dtype=torch.uint8, device="cuda")
big.fill_(1)
torch.cuda.synchronize()
timed("after 8 GB tensor")
env.close()
