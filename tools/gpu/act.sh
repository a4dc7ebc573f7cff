# fused act kernel: its tests, the S8 / learner / rollout tests, per-layer clock stamps, then an
# iteration kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8_act.py tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_rollout.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/act_tests.log 2>&1
rc=$?; tail -15 gpurun_out/act_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -f exp/libact_clock.so ]; then
  PYTHONPATH=.:tests:tools timeout -k 10 300 python -u tools/act_clock.py exp/libact_clock.so > gpurun_out/act_clock.log 2>&1 || exit $?
  tail -4 gpurun_out/act_clock.log
fi
bash tools/gpu/prof_iter.sh > /dev/null
