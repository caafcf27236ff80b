"""Step timeline from a rocprofv3 kernel trace: busy vs idle time between consecutive adamw launches (one per step),
and the largest idle gaps with the kernels around them.
usage: python scripts/timeline.py gpurun_out/prof_X/run_kernel_trace.csv [last_steps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
ad = [(i, dur(r)) for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
big = max(d for _, d in ad)
# one adamw launch per parameter group: step boundaries = the field group's (the long) launch
ends = [i for i, d in ad if d > big / 4]
seg = ends[-last - 1:]
lo, hi = seg[0] + 1, seg[-1]
ks = rows[lo:hi + 1]
t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
busy, gaps, prev = 0, [], None
for r in ks:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None and s > prev[0]:
        gaps.append((s - prev[0], prev[1], r["Kernel_Name"][:60]))
    busy += e - s
    prev = (max(e, prev[0]) if prev else e, r["Kernel_Name"][:60])
steps = len(seg) - 1
print(f"{steps} steps: span {(t1 - t0) / steps / 1e3:.3f} us/step... kernels {len(ks) / steps:.1f}/step, "
      f"busy {busy / steps / 1e3:.1f} us/step, idle {sum(g[0] for g in gaps) / steps / 1e3:.1f} us/step")
print(f"span per step {(t1 - t0) / steps / 1e6:.3f} ms")
for g in sorted(gaps, reverse=True)[:12]:
    print(f"  gap {g[0] / 1e3:8.1f} us after {g[1]} -> {g[2]}")

if len(sys.argv) > 3:
    # one step's launch sequence: gap before, duration, name
    a, b = seg[-2] + 1, seg[-1]
    prev_end = None
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e if prev_end is None else max(prev_end, e)
        print(f"{gap:7.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:110]}")
