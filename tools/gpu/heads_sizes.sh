set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/heads; rm -rf $O; mkdir -p $O
for b in ${BS:-1536 6144 24576 98304}; do for v in ${VARIANTS:-heads}; do
  B=$b LGX_MLP_LIB=$R/tools/exp/liblgx_mlp_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$b$v -- python3 $R/tools/heads_timing.py > $O/log_$b$v.txt 2>&1 || exit 1
  f=$(find $O/b$b$v -name "*kernel_stats.csv" | head -1)
  echo "== B=$b $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('head','aux','loss')): print('  ', r['Name'].split('(')[0][:40], r['Calls'], r['AverageNs'], r['MinNs'])
"
done; done
