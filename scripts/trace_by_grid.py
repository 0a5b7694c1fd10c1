"""Per-kernel, per-grid-size duration statistics from a rocprofv3 csv kernel trace
(`--kernel-trace --output-format csv`): bench.py also runs small helper envs (observation
statistics on one env) whose kernels share names with the workload's, so the workload's averages
are the rows of its grid size. Usage: trace_by_grid.py <dir with *kernel_trace.csv> <out.csv>"""
import collections
import csv
import glob
import statistics
import sys

root, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for path in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        if row.get("Grid_Size"):
            grid = int(float(row["Grid_Size"]))
        else:  # per-dimension columns
            grid = 1
            for d in "XYZ":
                grid *= int(float(row.get(f"Grid_Size_{d}", 1) or 1))
        acc[(name, grid)].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Grid_Size", "Calls", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
    for (name, grid), d in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, grid, len(d), round(sum(d) / len(d), 1), statistics.median(d), min(d), max(d)])
print(f"{len(acc)} (kernel, grid) groups -> {out}")
