# per-variant kernel stats of tools/gather_timing.py (one rocprofv3 run per variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/gather; rm -rf $O; mkdir -p $O
for v in ${VS:-a b c}; do
  V=$v PITCH=${PITCH:-628} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -- python3 $R/tools/gather_timing.py > $O/$v.log 2>&1 || exit 1
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'gather' in r['Name']: print('$v', r['Calls'], r['AverageNs'], r['MinNs'])
"
done
