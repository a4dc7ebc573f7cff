# GPU box: the whole -m gpu suite (verbose, per-test timeout), then one bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --timeout 180 --timeout-method thread ${TESTS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -1 gpurun_out/bench.log
fi
exit $rc
