set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -1 gpurun_out/bench.log
fi
exit $rc
