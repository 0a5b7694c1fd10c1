"""Merge gpurun_out/traffic_<tag>.json (scripts/pmc_summary.py: per workload key the HBM traffic per
launch, 2 x FETCH_SIZE + WRITE_SIZE with the gfx950 correction, the instruction counters, the
effective clock and the mean duration of the workload's own dispatches -- one instantiation and grid
per kernel base name) into profiles/traffic.json. The key's previous entries are REPLACED, not
updated, so no kernel of an older profile (or of another grid) survives under it.
With --only k1,k2 only those kernels of the key are replaced (a second profile of the same workload
for kernels the first one could not isolate, e.g. the episode-ahead generation in steady state).
Usage: traffic_merge.py <traffic_<tag>.json> <source note> [traffic.json] [--only k1,k2]"""
import json
import sys
from pathlib import Path

args = [a for a in sys.argv[1:] if not a.startswith("--only")]
only = next((a.split("=", 1)[1].split(",") for a in sys.argv[1:] if a.startswith("--only=")), None)
src, note = args[0], args[1]
out_path = Path(args[2] if len(args) > 2 else Path(__file__).resolve().parents[1] / "profiles" / "traffic.json")
new = json.loads(Path(src).read_text())
key = next(k for k in new if k not in ("counters", "clock_mhz"))
d = json.loads(out_path.read_text()) if out_path.exists() else {}
if only is None:
    d[key] = new[key]
    d.setdefault("counters", {})[key] = new["counters"][key]
    d.setdefault("clock_mhz", {})[key] = new["clock_mhz"][key]
    d.setdefault("sources", {})[key] = note
else:
    for sec, src_sec in ((d.setdefault(key, {}), new[key]), (d.setdefault("counters", {}).setdefault(key, {}), new["counters"][key]),
                         (d.setdefault("clock_mhz", {}).setdefault(key, {}), new["clock_mhz"][key])):
        for k in only:
            if k in src_sec:
                sec[k] = src_sec[k]
    d.setdefault("sources", {})[key] = d.get("sources", {}).get(key, "") + f"; {','.join(only)}: {note}"
out_path.write_text(json.dumps(d, indent=1) + "\n")
print(f"{key}: {len(new['counters'][key])} kernels -> {out_path}")
