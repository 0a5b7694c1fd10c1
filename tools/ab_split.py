"""A/B: C2 shape (8 x 64 x 5, ENVS envs) stepped as one env handle vs SPLIT handles of ENVS / SPLIT
envs each on their own HIP streams (one half's latency-bound step_a / step_c beside the other
half's issue-bound allocation). Env-only steps, episode-ahead demand, uniform[-1, 1] actions."""
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
STEPS = int(os.environ.get("STEPS", "1000"))
cfg = make_synthetic_env_config(8, 64, 5)
spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})


def run(split):
    n = E // split
    envs = [VecInventoryEnv(None, n, spec=spec, device=0, base_seed=1234, env_index_offset=i * n) for i in range(split)]
    streams = [torch.cuda.Stream() for _ in envs]
    acts = [torch.rand((n, 8, 5), device="cuda") * 2 - 1 for _ in envs]
    for x in envs:
        x.reset()
    torch.cuda.synchronize()

    def steps(k):
        main = torch.cuda.current_stream()
        for st in streams:
            st.wait_stream(main)
        for _ in range(k):
            for x, st, a in zip(envs, streams, acts):
                with torch.cuda.stream(st):
                    x.step(a)
        for st in streams:
            main.wait_stream(st)

    steps(1000)  # warm: episode-ahead demand in steady state
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(STEPS)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for x in envs:
        x.close()
    return dt / STEPS * 1e3


for split in [int(s) for s in os.environ.get("SPLITS", "1,2,1,2").split(",")]:
    ms = run(split)
    print(f"split {split}: {ms:.4f} ms/step, {E * 8 / ms / 1e3:.1f} M agent-steps/s", flush=True)
