"""Per-kernel GPU time over exactly one runner iteration of a rocprofv3 kernel trace (dev tool):
the span between two consecutive per-update row gathers. python tools/trace_iteration.py <trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, k in enumerate(ks) if "gather_rows" in k[2]]
a, b = marks[-2], marks[-1]
span = ks[b][0] - ks[a][0]
by = collections.Counter()
cnt = collections.Counter()
busy = 0
for s, e, n in ks[a:b]:
    key = n.split("(")[0][:70]
    by[key] += e - s
    cnt[key] += 1
    busy += e - s
print(f"iteration span {span / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms, {b - a} launches")
for k, v in by.most_common(25):
    print(f"{v / 1e6:8.3f} ms {cnt[k]:5d} x  {k}")
