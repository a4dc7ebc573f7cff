# single-problem S8 GEMM timings, product vs the variants in exp/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
PYTHONPATH=.:tools timeout -k 10 300 python -u tools/s8_one.py $(ls exp/*.so 2>/dev/null) > gpurun_out/s8_one.log 2>&1
rc=$?; tail -1 gpurun_out/s8_one.log; exit $rc
