set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_mlp.py > gpurun_out/bench_mlp.log 2>&1 && \
timeout -k 10 300 python tools/prof_learner.py > gpurun_out/prof_learner.log 2>&1
rc=$?
tail -12 gpurun_out/bench_mlp.log
exit $rc
