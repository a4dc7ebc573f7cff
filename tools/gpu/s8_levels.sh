# S8 minibatch launch-schedule experiment (tools/s8_levels.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
PYTHONPATH=.:tests timeout -k 10 400 python -u tools/s8_levels.py go2_c2 > gpurun_out/s8_levels.log 2>&1
rc=$?; head -30 gpurun_out/s8_levels.log; exit $rc
