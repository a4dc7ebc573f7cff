# The 256 x 256 kernel (exp/libs8_wide7.so: every kind routes its M, N >= 256 problems to it): S8
# kernel + executor tests with it in place of the product library (on the box's copy), then GEMM
# timings of the product and the variant in one process.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cp legged_gym_custom_amd/lib/liblgx_s8.so /tmp/liblgx_s8_product.so
cp exp/libs8_wide7.so legged_gym_custom_amd/lib/liblgx_s8.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s8_wide_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s8_wide_tests.log
cp /tmp/liblgx_s8_product.so legged_gym_custom_amd/lib/liblgx_s8.so
[ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 300 python -u tools/s8_bench.py --out gpurun_out/s8_bench.json --variants exp/libs8_wide7.so > gpurun_out/s8_bench.log 2>&1
rc=$?; tail -1 gpurun_out/s8_bench.log | cut -c1-400; exit $rc
