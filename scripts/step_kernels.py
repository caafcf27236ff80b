"""Per-step kernel table of graph-replayed training steps from a rocprofv3 kernel trace (two HIP streams aware).

Steps are delimited by the field group's AdamW launch (one per step).  Over the last N steps: wall span per step,
the summed kernel time per step (> span where the background stream overlaps the main one), and per kernel symbol
calls / step, average duration and ms / step.

usage: python scripts/step_kernels.py gpurun_out/prof_X/run_kernel_trace.csv [last_steps] [top] [skip_steps]

skip_steps drops that many step boundaries from the end first (e.g. the bench's secondary grid_raw5 steps).
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
ad = [(i, dur(r)) for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
big = max(d for _, d in ad)
ends = [i for i, d in ad if d > big / 4]
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ends = ends[:len(ends) - skip]
seg = ends[-last - 1:]
ks = rows[seg[0] + 1:seg[-1] + 1]
steps = len(seg) - 1
t0 = int(ks[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in ks)
# union of busy intervals (any stream) vs the summed durations
busy_union, cur_s, cur_e = 0, None, None
for r in ks:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy_union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy_union += cur_e - cur_s
summed = sum(dur(r) for r in ks)
print(f"{steps} graph-replayed steps: span {(t1 - t0) / steps / 1e6:.3f} ms/step, {len(ks) / steps:.1f} kernels/step, "
      f"summed kernel time {summed / steps / 1e6:.3f} ms/step, GPU busy (union over streams) "
      f"{busy_union / steps / 1e6:.3f} ms/step")
agg = collections.defaultdict(lambda: [0, 0])
for r in ks:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += dur(r)
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t / steps / 1e6:7.3f} ms/step {n / steps:6.1f} calls/step avg {t / n / 1e3:7.1f} us  {name[:110]}")
