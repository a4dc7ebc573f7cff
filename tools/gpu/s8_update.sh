# S8 core: kernel tests, S8 minibatch vs autograd path, learner goldens vs the reference, rollout
# graphs (incl. adaptation mode), RCCL all-reduce capture; then GEMM timings (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py tests/test_gpu_rollout.py tests/test_gpu_graph_allreduce.py -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/s8_update_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|worst|passed|failed|Error" gpurun_out/s8_update_tests.log | tail -70
PYTHONPATH=. timeout -k 10 300 python -u tools/s8_bench.py --out gpurun_out/s8_bench.json --variants exp/*.so > gpurun_out/s8_bench.log 2>&1
tail -3 gpurun_out/s8_bench.log
exit $rc
