#!/usr/bin/env python
"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv: python scripts/kstats.py <csv> <steps>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{len(rows)} kernel symbols, {tot / 1e6 / steps:.3f} ms of kernel time per step")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} ms/step {int(r['Calls']) / steps:6.1f} calls/step "
          f"avg {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:100]}")
