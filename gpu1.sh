set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python tools/bench_mlp.py > gpurun_out/bench_mlp.log 2>&1 && echo BENCHMLP_OK && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/bench.log 2>&1 && echo BENCH_OK
rc=$?
tail -15 gpurun_out/pytest_gpu.log; grep -v amdgpu gpurun_out/bench_mlp.log | tail -4; tail -1 gpurun_out/bench.log
exit $rc
