# learner tests + bench line (twice)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/learn; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/ab_knobs.sh "" 
