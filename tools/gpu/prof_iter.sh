set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_iter
mkdir -p $O
K=3 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/tools/prof_iter.py > $O/log.txt 2>&1
rc=$?
f=$(find $O -name "*_kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f 190 > $O/gaps.txt 2>&1
find $O -name "*_kernel_trace.csv" -delete
tail -2 $O/log.txt; head -50 $O/gaps.txt
exit $rc
