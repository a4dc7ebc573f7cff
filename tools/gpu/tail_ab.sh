# the heads-tail launch: S8 / learner tests, then the bench with it on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tail; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py --deselect "tests/test_gpu_learner_golden.py::test_gpu_adam_moments_after_update[go2_parkour_c4]" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu/ab_knobs.sh "" "LGX_HEADS_TAIL=0"
