"""Summarise rocprofv3 PMC csv passes per kernel (mean over dispatches)."""
import collections, csv, glob, sys
tag = sys.argv[1]
out = collections.defaultdict(dict)
for path in glob.glob(f"gpurun_out/pmc_*_{tag}/pmc_counter_collection.csv"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(path)):
        acc[row["Kernel_Name"].split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in acc.items():
        for c, x in v.items():
            out[k][c] = sum(x) / len(x)
for k, v in out.items():
    if "msc::" in k:
        print(k)
        for c in sorted(v):
            print(f"   {c:24s} {v[c]:.6g}")
