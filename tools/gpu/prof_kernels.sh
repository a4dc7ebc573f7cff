# rocprofv3 kernel stats of a short bench run: bash tools/gpu/prof_kernels.sh <tag> [env assignments...]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; shift
O=$R/gpurun_out/prof_$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --no_cpu_baseline --steps 4 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
f=$(find $O -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:110]}")
PY
