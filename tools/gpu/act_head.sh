# fused act head: the act / S8 / learner / rollout tests, an iteration kernel trace, a short bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8_act.py tests/test_gpu_s8.py tests/test_gpu_learner_golden.py tests/test_gpu_rollout.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/act_tests.log 2>&1
rc=$?; tail -15 gpurun_out/act_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/prof_iter.sh > /dev/null || exit $?
head -30 gpurun_out/prof_iter/gaps.txt
cd $R && timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/bench_head.log 2>&1
rc=$?; tail -1 gpurun_out/bench_head.log; exit $rc
