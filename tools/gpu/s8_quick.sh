# S8 kernel + executor tests, then a kernel trace of runner iterations (S8 update)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s8_quick.log 2>&1
rc=$?; tail -3 gpurun_out/s8_quick.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/prof_iter.sh
