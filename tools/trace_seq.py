"""Kernel sequence of one PPO minibatch and one rollout step from a rocprofv3 kernel trace
(dev tool): python tools/trace_seq.py <trace.csv>."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size_X", ""))
            for r in rows)


def show(a, b, t0):
    for s, e, n, g in ks[a:b + 1]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  grid={g:>8} {n.split('(')[0][:70]}")


idx = [i for i, k in enumerate(ks) if "tail_adam" in k[2]]
if len(idx) >= 3:
    print("---- minibatch")
    show(idx[-3] + 1, idx[-2], ks[idx[-3]][1])
idx = [i for i, k in enumerate(ks) if "env_step" in k[2]]
if len(idx) >= 3:
    print("---- rollout step")
    show(idx[-3], idx[-2], ks[idx[-3]][1])
