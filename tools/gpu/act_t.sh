set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8_act.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/act_tests.log 2>&1
rc=$?; grep -E "Mismatch|Greatest|passed|failed|Error" gpurun_out/act_tests.log | head -40; exit $rc
