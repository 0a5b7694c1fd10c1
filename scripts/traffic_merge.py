"""Merge gpurun_out/traffic_<tag>.json (scripts/pmc_summary.py: per workload key the HBM traffic per
launch, 2 x FETCH_SIZE + WRITE_SIZE with the gfx950 correction, the instruction counters, the
effective clock and the mean duration of the workload's own dispatches -- one instantiation and grid
per kernel base name) into profiles/traffic.json. The key's previous entries are REPLACED, not
updated, so no kernel of an older profile (or of another grid) survives under it.
Usage: traffic_merge.py <traffic_<tag>.json> <source note> [traffic.json]"""
import json
import sys
from pathlib import Path

src, note = sys.argv[1], sys.argv[2]
out_path = Path(sys.argv[3] if len(sys.argv) > 3 else Path(__file__).resolve().parents[1] / "profiles" / "traffic.json")
new = json.loads(Path(src).read_text())
key = next(k for k in new if k not in ("counters", "clock_mhz"))
d = json.loads(out_path.read_text()) if out_path.exists() else {}
d[key] = new[key]
d.setdefault("counters", {})[key] = new["counters"][key]
d.setdefault("clock_mhz", {})[key] = new["clock_mhz"][key]
d.setdefault("sources", {})[key] = note
out_path.write_text(json.dumps(d, indent=1) + "\n")
print(f"{key}: {len(new['counters'][key])} kernels -> {out_path}")
