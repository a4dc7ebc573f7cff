set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pr && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pr/trace -- python3 $R/tools/prof_rollout.py > $R/gpurun_out/pr/log 2>&1
rc=$?
find $R/gpurun_out/pr -name "*_kernel_trace.csv" -delete
exit $rc
