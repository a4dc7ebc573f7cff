set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lh; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -- python3 $R/tools/bench_loss_heads.py > $O/log.txt 2>&1 || exit $?
cd $R && python3 - <<'P'
import csv, glob, os
f = sorted(glob.glob("gpurun_out/lh/**/*kernel_trace.csv", recursive=True), key=os.path.getmtime)[-1]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for name in ("loss_heads_fwd", "loss_heads_bwd"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    h = len(d) // 2
    print(name, len(d), "first half %.2f us" % (sum(d[20:h]) / (h - 20)), "second half %.2f us" % (sum(d[h + 20:]) / (len(d) - h - 20)))
P
