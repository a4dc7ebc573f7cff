# rocprofv3 kernel stats of a short bench run: per-kernel calls / average us / share
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_bench; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no_cpu_baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
f=$(find $O/t -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; python3 $R/tools/trace_seq.py $(find $O/t -name "*kernel_trace.csv" | head -1) > $O/seq.txt 2>&1; find $O/t -name "*kernel_trace.csv" -delete
python3 - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:26]:
    print(f"{float(r['Percentage']):6.2f}%  {int(r['Calls']):6d}  {float(r['AverageNs'])/1000:8.1f} us  {r['Name'][:90]}")
PY
