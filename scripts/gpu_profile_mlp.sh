#!/bin/bash
# Kernel trace + PMC passes of the fused actor MLP alone (tools/bench_mlp.py, the bench's roofline_mlp
# launch): mean duration, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B) and MFMA busy cycles per
# launch -> gpurun_out/pmc_mlp_${TAG}.txt and gpurun_out/traffic_mlp_${TAG}.json.
set -u
TAG=${TAG:-r06}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp_$TAG -o trace --output-format csv -- python tools/bench_mlp.py > gpurun_out/bench_mlp_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcm_fetch_$TAG -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcm_write_$TAG -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/pmcm_sq_$TAG -o pmc --output-format csv -- python tools/bench_mlp.py > /dev/null 2>&1 || exit $?
python3 - "$TAG" > gpurun_out/pmc_mlp_$TAG.txt <<'EOF' || exit $?
import csv, glob, json, sys
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(list)
for p in glob.glob(f"gpurun_out/pmcm_*_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "mlp3_relu_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
v = {c: sum(x) / len(x) for c, x in acc.items()}
durs = []
for p in glob.glob(f"gpurun_out/prof_mlp_{tag}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "mlp3_relu_kernel" in r["Kernel_Name"]:
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
mean_ns = sum(durs) / len(durs)
traffic = int(round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024))
for c in sorted(v):
    print(f"{c:28s} {v[c]:.6g}")
print(f"dispatches {len(durs)}  mean duration {mean_ns / 1e3:.1f} us")
print(f"=> HBM traffic per launch {traffic / 1e6:.2f} MB (2 x FETCH + WRITE)")
json.dump({"traffic": traffic, "SQ_VALU_MFMA_BUSY_CYCLES": v.get("SQ_VALU_MFMA_BUSY_CYCLES"), "SQ_WAVES": v.get("SQ_WAVES"),
           "SQ_INSTS_VALU": v.get("SQ_INSTS_VALU"), "mean_ns": mean_ns},
          open(f"gpurun_out/traffic_mlp_{tag}.json", "w"), indent=1)
EOF
rm -rf gpurun_out/prof_mlp_$TAG gpurun_out/pmcm_*_$TAG
cat gpurun_out/pmc_mlp_$TAG.txt
