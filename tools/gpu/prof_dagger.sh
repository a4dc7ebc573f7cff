# rocprofv3 kernel stats of update_dagger graph replays (tools/prof_dagger.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_dagger; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REPS=${REPS:-5} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/prof_dagger.py > $O/out.txt 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
f=$(find $O -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
cat $O/out.txt
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:110]}")
PY
