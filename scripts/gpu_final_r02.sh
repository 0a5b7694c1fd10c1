#!/bin/bash
# Round-2 final evidence: GPU tests, smoke, default bench, C5 bench, rocprofv3 kernel stats + PMC
# of the env step (scripts/gpu_profile.sh), of the rollout, and of the fused MLP alone.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r02f}
if [ "${STAGE:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || exit $?
tail -n 2 gpurun_out/smoke_$T.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_$T.json.log | cut -c1-400
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5_$T.json.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_c5_$T.json.log | cut -c1-300
TAG=$T bash scripts/gpu_profile.sh > gpurun_out/profile_$T.log 2>&1 || exit $?
echo "env profile done"
fi
# the fused MLP alone: kernel stats + HBM bytes + MFMA busy cycles
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o trace --output-format csv -- python tools/bench_mlp.py > gpurun_out/bench_mlp_$T.log 2>&1 || exit $?
find gpurun_out/prof_mlp -name '*kernel_stats.csv' -exec cp {} gpurun_out/kernel_stats_mlp_$T.csv \;
# (one pass per TCC-heavy counter: FETCH_SIZE takes 3 of the 4 TCC counters, WRITE_SIZE 2)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_mlp1 -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_mlp3 -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmc_mlp2 -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
python3 - > gpurun_out/pmc_mlp_$T.txt <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_mlp*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mlp3_relu_kernel" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]][r.get("Dispatch_Id", "")].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    per = [sum(v) for v in d.values()]
    print(f"{k}: {sum(per)/len(per):.4g} per launch over {len(per)} launches")
PY
cat gpurun_out/pmc_mlp_$T.txt
rm -rf gpurun_out/prof_mlp gpurun_out/pmc_mlp1 gpurun_out/pmc_mlp2 gpurun_out/pmc_mlp3
# the MAPPO rollout: kernel stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roll -o trace --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --rollout-T 100 > gpurun_out/prof_roll_bench_$T.log 2>&1 || exit $?
find gpurun_out/prof_roll -name '*kernel_stats.csv' -exec cp {} gpurun_out/kernel_stats_roll_$T.csv \;
rm -rf gpurun_out/prof_roll
echo all done
