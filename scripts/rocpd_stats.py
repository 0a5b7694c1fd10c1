"""Per-kernel statistics from a rocprofv3 rocpd database (rocprofv3 -d DIR -o NAME writes
DIR/NAME_results.db): count, mean / total duration in microseconds, and (with --timeline N) the
dispatch timeline of the last N dispatches (start offset, duration, stream-queue).
Usage: python scripts/rocpd_stats.py gpurun_out/prof_c2/c2_results.db [--timeline 40] [--csv out.csv]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--skip-first", type=int, default=0, help="ignore the first N dispatches (warm-up)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end, queue_id from kernels order by start").fetchall()
    rows = rows[a.skip_first:]
    st = {}
    for n, s, e, q in rows:
        n = n.split("(")[0]
        d = st.setdefault(n, [0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1e3
    out = sorted(st.items(), key=lambda kv: -kv[1][1])
    lines = ["kernel,count,avg_us,total_us"] + [f"{k},{v[0]},{v[1] / v[0]:.2f},{v[1]:.1f}" for k, v in out]
    print("\n".join(lines))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")
    if a.timeline:
        t0 = rows[-a.timeline][1]
        for n, s, e, q in rows[-a.timeline:]:
            print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  q{q}  {n.split('(')[0][:60]}")


if __name__ == "__main__":
    main()
