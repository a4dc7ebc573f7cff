"""Mean PMC counter values per kernel over rocprofv3 --pmc passes (dev tool):
python pmc_summary.py <dir> [--by-grid]  (--by-grid: one entry per kernel and grid size, i.e. per
launch shape)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/*/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        key = r["Kernel_Name"].split("(")[0][-48:]
        if "--by-grid" in sys.argv:
            key += f" grid={r.get('Grid_Size', '?')}"
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "lgx" not in k and "env_step" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:32s} {sum(v) / len(v):14.0f}")
