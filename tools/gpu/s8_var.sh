# GEMM timings of the S8 build variants in exp/ (tools/s8_bench.py), then the PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/s8_bench.py --out gpurun_out/s8_bench.json --variants exp/*.so > gpurun_out/s8_bench.log 2>&1 || exit $?
tail -1 gpurun_out/s8_bench.log
[ -n "$NOPMC" ] && exit 0
bash tools/gpu/pmc_s8.sh > /dev/null
