# Kernel trace of K runner iterations after warm-up: busy/idle accounting (trace_gaps.py)
# and the kernel sequence of one minibatch and one rollout step (trace_seq.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_iter
rm -rf $O && mkdir -p $O
K=3 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/tools/prof_iter.py > $O/log.txt 2>&1
rc=$?
f=$(find $O -name "*_kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f 80 > $O/gaps.txt 2>&1
python3 $R/tools/trace_seq.py $f > $O/seq.txt 2>&1
python3 $R/tools/trace_outside.py $f > $O/outside.txt 2>&1
python3 $R/tools/trace_kernel_series.py $f env_step > $O/env_series.txt 2>&1
find $O -name "*_kernel_trace.csv" -delete
tail -2 $O/log.txt; head -40 $O/gaps.txt
exit $rc
