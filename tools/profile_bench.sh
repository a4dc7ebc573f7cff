# Bench-only round profile on the GPU box (the env kernel unchanged since profile_round.sh):
# kernel-trace stats of the bench command, then the default bench line (with cpu_baseline).
# Usage: bash tools/profile_bench.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_bench
rm -rf $O && mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 $R/bench.py --steps 5 --warmup 3 --no_cpu_baseline --kernel_iters 20 > $O/bench.log 2>&1 || exit $?
find $O -name "*_kernel_trace.csv" -delete
cd $R && timeout -k 10 400 python bench.py > $O/default.log 2>&1 || exit $?
tail -1 $O/bench.log; tail -1 $O/default.log
