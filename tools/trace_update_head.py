"""Kernels between the last rollout step and the first minibatch of a PPO update in a
rocprofv3 kernel trace (dev tool): python tools/trace_update_head.py <trace.csv> [n]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_max = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size_X", ""))
            for r in rows)
idx = [i for i, k in enumerate(ks) if "env_step" in k[2]]
last = idx[-1]
t0 = ks[last][1]
for s, e, name, g in ks[last + 1:last + 1 + n_max]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} grid={g:>8} {name.split('(')[0][:90]}")
