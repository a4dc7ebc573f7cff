# GPU check of the tree: the full -m gpu suite, the default bench line (with cpu_baseline),
# and the per-iteration GEMM census. Usage: bash tools/gpu/run_suite.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
[ -n "$NOCENSUS" ] && exit 0
timeout -k 10 200 python tools/gemm_census.py > $O/census.log 2>&1 || exit $?
head -12 $O/census.log
