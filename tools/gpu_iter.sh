# GPU dev loop (run on the box): learner/MLP GPU tests, a bench line, and a kernel trace of
# three runner iterations summarised by trace_gaps.py / trace_seq.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_mlp.py tests/test_gpu_learner.py} > $O/t1.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > $O/bench.log 2>&1
rc=$?; echo bench rc=$rc; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NOPROF" ] && exit 0
rm -rf $O/prof_iter2; mkdir -p $O/prof_iter2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_iter2/trace -- python3 $R/tools/prof_iter.py > $O/prof_iter2/log.txt 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
cd $R && T=$(find $O/prof_iter2 -name "*kernel_trace.csv") && python3 tools/trace_gaps.py $T 60 > $O/prof_iter2/gaps.txt && python3 tools/trace_seq.py $T > $O/prof_iter2/seq.txt
head -16 $O/prof_iter2/gaps.txt
