"""Turn rocprofv3 CSVs (from tools/profile_round.sh) into the committed profile files:
  <out>/<tag>_bench_kernel_stats.csv   kernel-trace --stats of the bench command
  <out>/<tag>_env_traffic.json         env-step kernel HBM traffic per launch from PMC
Traffic per MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE from separate --pmc
passes, in KiB; FETCH_SIZE doubled (gfx950 tallies 128-B read requests at 64 B)."""
import csv
import glob
import json
import os
import shutil
import sys

src, out, tag = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(out, exist_ok=True)
stats = glob.glob(os.path.join(src, "trace", "*", "*_kernel_stats.csv"))
if stats:
    shutil.copy(stats[0], os.path.join(out, f"{tag}_bench_kernel_stats.csv"))
for sub, name in (("parkour", "parkour_n8192"), ("anymal", "anymal_rough_n4096")):
    st = glob.glob(os.path.join(src, sub, "*", "*_kernel_stats.csv"))
    if st:
        shutil.copy(st[0], os.path.join(out, f"{tag}_env_{name}_kernel_stats.csv"))


def pmc(name):
    f = glob.glob(os.path.join(src, name, "*", "*_counter_collection.csv"))
    vals = {}
    for r in csv.DictReader(open(f[0])):
        if "env_step_kernel" in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return vals


res = {"kernel": "lgx::env_step_kernel<true, false>", "workload": "go2 flat, 4096 envs, actions N(0,1) clipped"}
fetch = pmc("fetch").get("FETCH_SIZE", [])
write = pmc("write").get("WRITE_SIZE", [])
if fetch and write:
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res.update({"launches": len(fetch), "FETCH_SIZE_KiB_raw": f_kib, "WRITE_SIZE_KiB": w_kib,
                "fetch_bytes_corrected": 2 * f_kib * 1024, "write_bytes": w_kib * 1024,
                "traffic_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
                "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes"})
json.dump(res, open(os.path.join(out, f"{tag}_env_traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
