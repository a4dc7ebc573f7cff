# kernel-time stats of tools/heads_timing.py for the product library and each variant
# (VARIANTS="a b": tools/exp/liblgx_mlp_<v>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/heads; rm -rf $O; mkdir -p $O
for v in product $VARIANTS; do
  lib=$R/tools/exp/liblgx_mlp_$v.so; [ $v = product ] && lib=$R/legged_gym_custom_amd/lib/liblgx_mlp.so
  LGX_MLP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -- python3 $R/tools/heads_timing.py > $O/log_$v.txt 2>&1 || exit 1
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('head','aux','loss')): print('  ', r['Name'].split('(')[0][:40], r['Calls'], r['AverageNs'], r['MinNs'])
"
done
