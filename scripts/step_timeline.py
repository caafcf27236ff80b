import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 25
dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
ad = [(i, dur(r)) for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
big = max(d for _, d in ad)
ends = [i for i, d in ad if d > big / 4]
if skip: ends = ends[:-skip]
seg = ends[-3:]
lo, hi = seg[0] + 1, seg[1]
ks = rows[lo:hi + 1]
t0 = int(ks[0]["Start_Timestamp"])
print("one step, span %.1f us" % ((int(ks[-1]["End_Timestamp"]) - t0) / 1e3))
for r in ks:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3; e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"q{r['Queue_Id']:>2} {s:8.1f} {e:8.1f} {e-s:7.1f}  {r['Kernel_Name'][:90]}")
