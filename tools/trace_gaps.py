"""Busy/idle accounting of a rocprofv3 kernel trace (dev tool): python trace_gaps.py <trace.csv> [last_ms].
Looks at the last `last_ms` of the trace: kernel time per name and the idle gaps between
consecutive kernels (a launch-bound stream shows many small gaps)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 200.0
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
t_end = ks[-1][1]
ks = [k for k in ks if k[0] >= t_end - last_ms * 1e6]
span = ks[-1][1] - ks[0][0]
busy = 0
gaps = []
prev_end = ks[0][0]
by = collections.Counter()
cnt = collections.Counter()
for s, e, n in ks:
    busy += e - s
    gaps.append(max(0, s - prev_end))
    prev_end = max(prev_end, e)
    key = n.split("(")[0][:80]
    by[key] += e - s
    cnt[key] += 1
print(f"kernels {len(ks)} span {span / 1e6:.2f} ms busy {busy / 1e6:.2f} ms idle {(span - busy) / 1e6:.2f} ms")
gs = sorted(gaps)
print("gap us: median %.2f p90 %.2f max %.1f; gaps > 20us: %d totalling %.2f ms" % (
    gs[len(gs) // 2] / 1e3, gs[int(len(gs) * 0.9)] / 1e3, gs[-1] / 1e3, sum(g > 20000 for g in gs),
    sum(g for g in gs if g > 20000) / 1e6))
for k, v in by.most_common(40):
    print(f"{v / 1e6:8.3f} ms {cnt[k]:6d} x {v / cnt[k] / 1e3:8.2f} us  {k}")
