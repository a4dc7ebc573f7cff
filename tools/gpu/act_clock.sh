set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
PYTHONPATH=.:tests:tools timeout -k 10 300 python -u tools/act_clock.py exp/libact_clock.so > gpurun_out/act_clock.log 2>&1
rc=$?; tail -5 gpurun_out/act_clock.log; exit $rc
