#!/bin/bash
# Kernel timeline of the pipelined env step (rocprofv3 --kernel-trace): the demand kernel of step t+1
# on the library's side stream against step t's phase kernels; prints per-step periods and the gaps
# between the two chains. usage: [ARGS="..."] [OUT=trace_env] bash scripts/gpu_trace_env.sh
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
out=${OUT:-trace_env}
ARGS=${ARGS:-"--steps 60 --warmup 10 --no-cpu-baseline --rollout-T 0 --c2-envs 0 --c5-envs 0 --no-ea-line"}
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/$out -o trace --output-format csv -- python bench.py $ARGS > gpurun_out/${out}_bench.log 2>&1 || exit $?
f=$(find gpurun_out/$out -name '*kernel_trace.csv' | head -1)
python3 - "$f" > gpurun_out/${out}_summary.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    for k in ("demand_v3", "demand_unit", "demand_v2", "alloc_lane", "alloc_scan", "step_a", "step_b", "step_c", "alloc_sort", "reset", "ea_materialize"):
        if k in n: return k
    return n[:30]
big = [r for r in rows if int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0) >= 32768 * 4 or "alloc_lane" in r["Kernel_Name"]]
sel = big[-240:]
t0 = int(sel[0]["Start_Timestamp"])
for r in sel:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{short(r['Kernel_Name']):14s} q{r.get('Queue_Id', '?'):>3s} {s:10.1f} {e:10.1f} {e - s:8.1f}")
PY
rm -rf gpurun_out/$out
head -3 gpurun_out/${out}_summary.txt
