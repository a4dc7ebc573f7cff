# S8 GEMM core: GPU tests + timing against the fp32-operand GEMMs (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_s8.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s8_tests.log 2>&1
rc=$?
tail -30 gpurun_out/s8_tests.log
[ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 300 python -u tools/s8_bench.py --out gpurun_out/s8_bench.json --variants exp/*.so > gpurun_out/s8_bench.log 2>&1
rc=$?
tail -5 gpurun_out/s8_bench.log
exit $rc
