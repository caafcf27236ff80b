#!/usr/bin/env python
"""Per-kernel totals and GPU busy/idle split from a rocprofv3 --kernel-trace CSV.

    python scripts/trace_summary.py gpurun_out/prof_fast/run_kernel_trace.csv --steps 25 [--tail-frac 0.8]

--tail-frac keeps the last fraction of dispatches (skip warm-up); busy = union of kernel intervals.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=1.0, help="steps covered by the kept dispatches")
    ap.add_argument("--tail-frac", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * (1 - a.tail_frac)):]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    span = iv[-1][1] - iv[0][0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "<" in short and "gemm_kernel" not in short:
            short = short.split("<")[0] + "<..>"
        per[short][0] += 1
        per[short][1] += e - s
    st = a.steps
    print(f"dispatches {len(iv)} ({len(iv) / st:.0f}/step); span {span / 1e6 / st:.3f} ms/step; "
          f"busy {busy / 1e6 / st:.3f} ms/step ({100 * busy / span:.1f}%); idle {(span - busy) / 1e6 / st:.3f} ms/step")
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e6 / st:8.3f} ms/step {n / st:7.1f}/step {t / n / 1e3:9.1f} us  {k[:90]}")


if __name__ == "__main__":
    main()
