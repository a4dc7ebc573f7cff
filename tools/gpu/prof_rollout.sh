set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_rollout
mkdir -p $O
K=10 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 $R/tools/prof_rollout.py > $O/log.txt 2>&1
rc=$?
find $O -name "*_kernel_trace.csv" -delete
tail -3 $O/log.txt
exit $rc
