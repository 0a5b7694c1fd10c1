"""Summarise rocprofv3 PMC csv passes per kernel (mean over dispatches) and write the per-launch
HBM traffic of the env kernels to gpurun_out/traffic_<tag>.json.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): MI355X_MICROARCH.md "HBM [CDNA4]" -- on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (TCC_EA0_RDREQ x 64 B), WRITE_SIZE is
exact for 16-B-per-lane stores."""
import collections
import csv
import glob
import json
import re
import sys

tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "8x64x5x32768"
out = collections.defaultdict(dict)
# dispatches are grouped by kernel and grid size; per kernel only the largest grid (the workload's
# launches, not those of the small helper envs bench.py builds, e.g. for observation statistics)
grids = collections.defaultdict(set)
for path in glob.glob(f"gpurun_out/pmc_*_{tag}/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0]
        grid = int(float(row.get("Grid_Size", 0) or 0))
        grids[name].add(grid)
        acc[(name, grid)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for (name, grid), v in acc.items():
        if grid != max(grids[name]):
            continue
        for c, x in v.items():
            out[name][c] = sum(x) / len(x)
        out[name]["grid_size"] = grid
traffic = {}
counters = {}
for k, v in sorted(out.items()):
    if "msc::" not in k:
        continue
    print(k)
    for c in sorted(v):
        print(f"   {c:24s} {v[c]:.6g}")
    m = re.search(r"msc::(\w+)", k)
    if m and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        traffic[m.group(1)] = int(round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024))
        print(f"   => HBM traffic per launch {traffic[m.group(1)] / 1e6:.2f} MB (2 x FETCH + WRITE)")
    if m:
        counters[m.group(1)] = {c: v[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES") if c in v}
# effective shader clock per kernel: GRBM_GUI_ACTIVE counts busy cycles summed over the 8 XCDs
# (MI355X_MICROARCH.md), divided by the kernel's mean duration at the same grid (kernel trace)
clocks = {}
dur = {}
try:
    for row in csv.DictReader(open(f"gpurun_out/kernel_stats_by_grid_{tag}.csv")):
        name = row["Name"].split("(")[0]
        g = int(row["Grid_Size"])
        if name not in dur or g > dur[name][0]:
            dur[name] = (g, float(row["AverageNs"]))
except FileNotFoundError:
    pass
for k, v in out.items():
    m = re.search(r"msc::(\w+)", k)
    if m and "GRBM_GUI_ACTIVE" in v and k in dur and dur[k][1] > 0:
        clocks[m.group(1)] = round(v["GRBM_GUI_ACTIVE"] / 8 / dur[k][1] * 1e3, 1)  # MHz
        print(f"{k}: effective clock {clocks[m.group(1)]} MHz (GRBM_GUI_ACTIVE / 8 / {dur[k][1] / 1e3:.1f} us)")
json.dump({workload: traffic, "counters": {workload: counters}, "clock_mhz": {workload: clocks}},
          open(f"gpurun_out/traffic_{tag}.json", "w"), indent=1)
