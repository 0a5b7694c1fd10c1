"""The rollout's fused actor MLP alone (msc_mlp3_relu_forward, csrc/mlp.hip) at the C3 MAPPO shape:
34 -> 256 -> 256 -> 5 over E x W = 262,144 rows, REPS launches timed with HIP events on the launch
stream. Used under rocprofv3 (kernel stats / PMC) so that the profiler's average for
mlp3_relu_kernel is the same launch bench.py reports as roofline_mlp."""
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "marl-sc_amd"))
import torch  # noqa: E402

from marlsc.mlp import mlp3_forward  # noqa: E402
from marlsc.rollout import MLP  # noqa: E402

N = int(os.environ.get("ROWS", str(32768 * 8)))
L, H, KO = 34, 256, 5
REPS = int(os.environ.get("REPS", "50"))
torch.manual_seed(0)
mlp = MLP(L, KO, {"hidden_sizes": [H, H]}).cuda()
mods = list(mlp)
x = torch.randn(N, L, device="cuda")
y = torch.empty(N, KO, device="cuda")
with torch.no_grad():
    for _ in range(3):
        mlp3_forward(mods, x, out=y)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(REPS):
        mlp3_forward(mods, x, out=y)
    b.record()
    torch.cuda.synchronize()
    ref = mods[4](torch.relu(mods[2](torch.relu(mods[0](x[:4096])))))
t = a.elapsed_time(b) / 1e3 / REPS
fl = 2.0 * N * (L * H + H * H + H * KO)
err = float((y[:4096] - ref).abs().max())
print(json.dumps({"kernel": "mlp3_relu_kernel", "rows": N, "ms": round(t * 1e3, 4), "tflops": round(fl / t / 1e12, 2),
                  "frac_f32_mfma_peak": round(fl / t / 1e12 / 157.3, 4), "max_abs_err_vs_torch": err}))
