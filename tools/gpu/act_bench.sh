set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
PYTHONPATH=.:tests:tools timeout -k 10 300 python -u tools/act_bench.py $(ls exp/libact_*.so 2>/dev/null) > gpurun_out/act_bench.log 2>&1
rc=$?; tail -2 gpurun_out/act_bench.log; exit $rc
