#!/bin/bash
# C5 line (2 reps) and step_b in-kernel counters (prof build) at C5. Stops at the first failure.
set -u
TAG=${1:-c5p}
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 300 python bench.py --config c5 --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_${TAG}_$rep.json.log 2>&1
rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/bench_${TAG}_$rep.json.log') if l.startswith('{')][0];print('C5', round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms'])"
done
timeout -k 10 200 python tools/prof_step_b.py > gpurun_out/prof_step_b_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_step_b_${TAG}.log; exit $rc
