#!/bin/bash
# Kernel timeline of the MAPPO rollout (rocprofv3 --kernel-trace): per-step ordering of the
# pipelined demand kernel against the step chain and the policy kernels.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline --rollout-T 100 --c2-envs 0 --c5-envs 0 --no-ea-line"}
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/trace_roll -o trace --output-format csv -- python bench.py $ARGS > gpurun_out/trace_roll_bench.log 2>&1 || exit $?
f=$(find gpurun_out/trace_roll -name '*kernel_trace.csv' | head -1)
python3 - "$f" > gpurun_out/trace_roll_summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    for k in ("demand_v3", "demand_unit", "alloc_lane", "step_a", "step_c", "mlp3_relu_kernel<8", "mlp3_relu_kernel<2", "mlp2_relu", "meanstd", "obs_filter", "gae4", "gauss", "Cijk", "elementwise", "reduce"):
        if k in n: return k
    return n[:30]
# last 400 kernels: print name, start (us rel), end, queue id
t0 = int(rows[-400]["Start_Timestamp"])
for r in rows[-400:]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{short(r['Kernel_Name']):24s} q{r.get('Queue_Id', '?'):>3s} {s:10.1f} {e:10.1f} {e - s:8.1f}")
PY
rm -rf gpurun_out/trace_roll
head -5 gpurun_out/trace_roll_summary.txt
