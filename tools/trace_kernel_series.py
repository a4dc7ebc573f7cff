"""Durations of every launch of one kernel, in trace order (dev tool):
python tools/trace_kernel_series.py <trace.csv> <name substring>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
sel = [(s, e) for s, e, n in ks if sys.argv[2] in n]
t0 = sel[0][0]
for i, (s, e) in enumerate(sel):
    print(f"{i:4d} t={(s - t0) / 1e3:10.1f} us  dur={(e - s) / 1e3:7.1f} us")
