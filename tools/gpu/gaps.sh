set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gaps
rm -rf $O && mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/bench.py --steps 4 --warmup 2 --no_cpu_baseline --kernel_iters 5 > $O/bench.log 2>&1 || exit $?
f=$(find $O -name "*_kernel_trace.csv" | head -1)
cd $R && python tools/trace_gaps.py $f 100 > $O/gaps.txt && python tools/trace_iteration.py $f > $O/iter.txt
find $O -name "*_kernel_trace.csv" -delete
cat $O/gaps.txt | head -12; cat $O/iter.txt | head -5
