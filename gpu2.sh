set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pb && cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pb/trace -- python3 $R/bench.py --steps 5 --warmup 3 --no_cpu_baseline --kernel_iters 20 > $R/gpurun_out/pb/bench.log 2>&1
rc=$?
find $R/gpurun_out/pb -name "*_kernel_trace.csv" -delete
tail -1 $R/gpurun_out/pb/bench.log
exit $rc
