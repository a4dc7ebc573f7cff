# Device time of the learner's small GEMM shapes alone (rocprofv3 kernel trace).
# Usage: bash tools/gpu/small_gemm.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/small_gemm
rm -rf $O && mkdir -p $O && cd /tmp && export TMPDIR=/tmp
for spec in "128,12:fwd" "128,12:dx" "64,20:fwd" "128,64:fwd" "512,256:fwd" "736,512:fwd"; do
  sh=${spec%%:*}; md=${spec##*:}
  SHAPE=$sh MODE=$md IT=40 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$md_$sh -o run -- python3 $R/tools/gemm_one.py > $O/log_${md}_${sh}.txt 2>&1 || exit $?
  f=$(find $O/$md_$sh -name "*kernel_stats.csv" | head -1)
  echo "== $md $sh"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'gemm' in r['Name'] or 'elementwise' in r['Name']: print(f\"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.2f} us {r['Name'][:80]}\")
"
done
