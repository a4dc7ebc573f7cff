set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_learner.py > gpurun_out/mlp_tests.log 2>&1
rc=$?
tail -5 gpurun_out/mlp_tests.log
[ $rc -eq 0 ] && timeout -k 10 120 python tools/bench_mlp.py 2>&1 | grep -v amdgpu.ids
exit $rc
