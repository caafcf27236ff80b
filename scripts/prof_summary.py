#!/usr/bin/env python
"""Summarise a rocprofv3 rocpd database (kernel dispatches) as a per-kernel stats table.

    python scripts/prof_summary.py gpurun_out/prof2/run_results.db [--steps K] [--by-grid] [--csv out.csv]
"""
import argparse
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps (ms/step column)")
    ap.add_argument("--by-grid", action="store_true", help="split kernels by grid size")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    gx = "grid_x" if "grid_x" in cols else None
    key = "name" + (", grid_x, grid_z" if a.by_grid and gx else "")
    rows = con.execute(f"select {key}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                       f"from kernels group by {key} order by sum(end-start) desc").fetchall()
    total = sum(r[-4] for r in rows)
    out = []
    hdr = ["kernel"] + (["grid_x", "grid_z"] if a.by_grid and gx else []) + \
          ["calls", "total_ms", "avg_us", "min_us", "max_us", "pct"] + (["ms_per_step"] if a.steps else [])
    for r in rows:
        k = list(r[:-5])
        n, tot, avg, mn, mx = r[-5:]
        rec = k + [n, tot / 1e6, avg / 1e3, mn / 1e3, mx / 1e3, 100.0 * tot / total]
        if a.steps:
            rec.append(tot / 1e6 / a.steps)
        out.append(rec)
    if a.csv:
        import csv
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            w.writerows(out)
    for rec in out[:a.top]:
        name = str(rec[0])
        name = name if len(name) < 70 else name[:67] + "..."
        print(f"{name:70s} " + " ".join(f"{v:10.3f}" if isinstance(v, float) else f"{v:>8}" for v in rec[1:]))
    print(f"total kernel time {total / 1e6:.3f} ms over {sum(r[-5] for r in rows)} dispatches", file=sys.stderr)


if __name__ == "__main__":
    main()
