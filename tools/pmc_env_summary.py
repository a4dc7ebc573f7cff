"""Summarise tools/gpu/pmc_env.sh: per-launch means of every counter for the Go2 env-step
kernel, the dword-access FETCH/WRITE calibration, and the HBM traffic per launch with the
calibrated correction. Writes gpurun_out/pmc_env_<tag>/{<tag>_env_kernel_pmc.txt,
<tag>_env_traffic.json} (copied into profiles/ by hand)."""
import collections
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
CALIB_BYTES = 512 << 20
TASK = os.environ.get("TASK", "go2")
N = int(os.environ.get("N", "4096"))
# bench.py reads the newest <round>_env_kernel_pmc.txt / <round>_env_traffic.json (the Go2 bench
# workload); the other tasks' files carry the task name so they never match those globs
STEM = f"{tag}_env" if TASK == "go2" else f"{tag}_env_{TASK}"


def counters(sub, match):
    acc = collections.defaultdict(list)
    names = set()
    for f in glob.glob(os.path.join(src, sub, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                names.add(r["Kernel_Name"])
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}, names


env = {}
kname = None
for p in sorted(glob.glob(os.path.join(src, "p*"))):
    if not os.path.isdir(p):
        continue
    vals, _, names = counters(os.path.basename(p), "env_step_kernel")
    env.update(vals)
    kname = kname or next(iter(names), None)
cal = {}
for sub, ctr in (("c1", "FETCH_SIZE"), ("c2", "WRITE_SIZE")):
    for kern in ("read_dword(", "read_dwordx4", "write_dword"):
        vals, _, _ = counters(sub, kern)
        if ctr in vals:
            cal[f"{kern.strip('(')}:{ctr}"] = vals[ctr] * 1024 / CALIB_BYTES
lines = [f"# rocprofv3 --pmc passes over tools/env_kernel_driver.py ({TASK}, {N} envs): per-launch means; kernel {kname}",
         "# (SQ_* cycle counters in quad-cycles). Calibration (tools/calib/hbm_calib, 512 MiB, counter bytes / true bytes):"]
lines += [f"#   {k:28s} {v:.3f}" for k, v in sorted(cal.items())]
for k in sorted(env):
    lines.append(f"   {k:36s} {env[k]:16.0f}")
if "SQ_WAVE_CYCLES" in env:
    lines.append(f"   wait fraction SQ_WAIT_ANY/SQ_WAVE_CYCLES = {env.get('SQ_WAIT_ANY', 0) / env['SQ_WAVE_CYCLES']:.3f}")
    lines.append(f"   VALU instructions per env step = {env.get('SQ_INSTS_VALU', 0) / N:.0f}, SALU {env.get('SQ_INSTS_SALU', 0) / N:.0f}, LDS {env.get('SQ_INSTS_LDS', 0) / N:.0f}")
txt = "\n".join(lines)
open(os.path.join(src, f"{STEM}_kernel_pmc.txt"), "w").write(txt + "\n")
print(txt)
fr = cal.get("read_dword:FETCH_SIZE")
wr = cal.get("write_dword:WRITE_SIZE")
if "FETCH_SIZE" in env and "WRITE_SIZE" in env and fr and wr:
    res = {"kernel": kname, "workload": f"{TASK}, {N} envs, actions N(0,1) clipped (tools/env_kernel_driver.py)",
           "FETCH_SIZE_KiB_raw": env["FETCH_SIZE"], "WRITE_SIZE_KiB_raw": env["WRITE_SIZE"],
           "calibration": {"dword_read_fetch_ratio": fr, "dword_write_ratio": wr,
                           "dwordx4_read_fetch_ratio": cal.get("read_dwordx4:FETCH_SIZE")},
           "fetch_bytes_corrected": env["FETCH_SIZE"] * 1024 / fr, "write_bytes": env["WRITE_SIZE"] * 1024 / wr}
    res["traffic_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
    res["correction"] = ("counter KiB -> bytes, divided by the counter/true ratio measured on dword-per-lane "
                         "coalesced reads and writes of a 512 MiB buffer (tools/calib/hbm_calib.hip)")
    json.dump(res, open(os.path.join(src, f"{STEM}_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))
