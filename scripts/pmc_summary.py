"""Summarise rocprofv3 PMC csv passes per kernel (mean over dispatches) and write the per-launch
HBM traffic of the env kernels to gpurun_out/traffic_<tag>.json.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): MI355X_MICROARCH.md "HBM [CDNA4]" -- on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (TCC_EA0_RDREQ x 64 B), WRITE_SIZE is
exact for 16-B-per-lane stores.

Only the workload's dispatches count. bench.py also runs small helper envs (observation statistics
on one env) whose kernels share base names -- and sometimes template instantiations -- with the
workload's, so dispatches are grouped by (kernel, grid size) and a group belongs to the workload
only if its grid has at least E threads (E = the workload key's env count: every per-env kernel
launches >= 1 thread per env; the one-block order-count sort is the exception). Each base name
(template arguments stripped; the episode-ahead demand instantiation kept apart as *_ea) must then
map to exactly one (instantiation, grid), which is what traffic_merge.py keys the JSON by.
Usage: pmc_summary.py <tag> <workload key WxRxKxE>"""
import collections
import csv
import glob
import json
import os
import re
import sys

tag = sys.argv[1]
workload = sys.argv[2] if len(sys.argv) > 2 else "8x64x5x32768"
E = int(workload.split("x")[-1])


def base_name(full: str) -> str:
    m = re.search(r"msc::(\w+)(?:<(.*)>)?", full)
    if not m:
        return ""
    name = m.group(1)
    if name.startswith("demand_") and (m.group(2) or "").replace(" ", "").endswith(",true"):
        name += "_ea"
    return name


def workload_grid(name: str, grid: int) -> bool:
    return grid >= E or "alloc_sort_kernel" in name


acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"gpurun_out/pmc_*_{tag}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0]
        grid = int(float(row.get("Grid_Size", 0) or 0))
        if "msc::" not in name or not workload_grid(name, grid):
            continue
        acc[(name, grid)][row["Counter_Name"]].append(float(row["Counter_Value"]))
# one (instantiation, grid) per base name: the one with the most dispatches (the workload's steady
# state: e.g. the episode-ahead refill launches rather than the one bulk launch that fills the slots
# at the start), the larger grid on ties
def n_disp(key):
    return max(len(x) for x in acc[key].values())


chosen = {}
for (name, grid) in acc:
    b = base_name(name)
    if b in chosen and chosen[b] != (name, grid):
        old = chosen[b]
        print(f"# note: {b}: several workload-sized groups {old} ({n_disp(old)} dispatches) / {(name, grid)} "
              f"({n_disp((name, grid))}); keeping the one with more dispatches", file=sys.stderr)
        if (n_disp((name, grid)), grid) <= (n_disp(old), old[1]):
            continue
    chosen[b] = (name, grid)
only = [x for x in os.environ.get("PMC_ONLY", "").split(",") if x]
if only:
    chosen = {b: v for b, v in chosen.items() if b in only}
traffic, counters, clocks = {}, {}, {}
dur = {}
try:
    for row in csv.DictReader(open(f"gpurun_out/kernel_stats_by_grid_{tag}.csv")):
        name = row["Name"].split("(")[0]
        g = int(row["Grid_Size"])
        if (name, g) in acc:
            dur[(name, g)] = float(row["AverageNs"])
except FileNotFoundError:
    pass
for b, (name, grid) in sorted(chosen.items()):
    v = {c: sum(x) / len(x) for c, x in acc[(name, grid)].items()}
    v["grid_size"] = grid
    v["dispatches"] = n_disp((name, grid))
    print(f"{name}")
    for c in sorted(v):
        print(f"   {c:24s} {v[c]:.6g}")
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        traffic[b] = int(round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024))
        print(f"   => HBM traffic per launch {traffic[b] / 1e6:.2f} MB (2 x FETCH + WRITE)")
    counters[b] = {c: v[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES",
                                     "SQ_LDS_BANK_CONFLICT", "grid_size", "dispatches") if c in v}
    # effective shader clock: GRBM_GUI_ACTIVE counts busy cycles summed over the 8 XCDs
    # (MI355X_MICROARCH.md), divided by the kernel's mean duration at the same grid (kernel trace)
    d = dur.get((name, grid), 0.0)
    if "GRBM_GUI_ACTIVE" in v and d > 0:
        clocks[b] = round(v["GRBM_GUI_ACTIVE"] / 8 / d * 1e3, 1)  # MHz
        print(f"{name}: effective clock {clocks[b]} MHz (GRBM_GUI_ACTIVE / 8 / {d / 1e3:.1f} us)")
    if d > 0:
        counters[b]["mean_ns"] = d
json.dump({workload: traffic, "counters": {workload: counters}, "clock_mhz": {workload: clocks}},
          open(f"gpurun_out/traffic_{tag}.json", "w"), indent=1)
