"""Merge a PMC summary (scripts/pmc_summary.py output, gpurun_out/pmc_summary_<tag>.txt) into
profiles/traffic.json under a workload key: per kernel the HBM traffic per launch (2 x FETCH_SIZE +
WRITE_SIZE, KiB -> B, MI355X_MICROARCH.md gfx950 correction), the instruction counters and the
effective clock (GRBM_GUI_ACTIVE / 8 / mean duration). The episode-ahead instantiation of the
demand kernel is kept apart as demand_unit_kernel_ea.
Usage: traffic_merge.py <pmc_summary.txt> <workload key> <source note> [traffic.json]"""
import json
import re
import sys
from pathlib import Path

src, key, note = sys.argv[1], sys.argv[2], sys.argv[3]
out_path = Path(sys.argv[4] if len(sys.argv) > 4 else Path(__file__).resolve().parents[1] / "profiles" / "traffic.json")
kern, vals, clocks = None, {}, {}
for line in open(src):
    m = re.match(r"^(?:void )?msc::(\w+)(?:<(.*)>)?\s*$", line.rstrip())
    if m:
        name = m.group(1)
        if name == "demand_unit_kernel" and (m.group(2) or "").replace(" ", "").endswith(",true"):
            name += "_ea"
        kern = name
        vals[kern] = {}
        continue
    m = re.match(r"^(?:void )?msc::(\w+)(?:<(.*)>)?: effective clock ([\d.]+) MHz", line)
    if m:
        name = m.group(1)
        if name == "demand_unit_kernel" and (m.group(2) or "").replace(" ", "").endswith(",true"):
            name += "_ea"
        clocks[name] = float(m.group(3))
        continue
    m = re.match(r"^\s+(\w+)\s+([-\d.e+]+)\s*$", line)
    if m and kern:
        vals[kern][m.group(1)] = float(m.group(2))
d = json.loads(out_path.read_text()) if out_path.exists() else {}
d.setdefault(key, {})
d.setdefault("counters", {}).setdefault(key, {})
d.setdefault("clock_mhz", {}).setdefault(key, {})
for k, v in vals.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        d[key][k] = int(round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024))
    d["counters"][key][k] = {c: v[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES",
                                               "SQ_LDS_BANK_CONFLICT", "grid_size") if c in v}
d["clock_mhz"][key].update(clocks)
d.setdefault("sources", {})[key] = note
out_path.write_text(json.dumps(d, indent=1) + "\n")
print(f"{key}: {len(vals)} kernels -> {out_path}")
