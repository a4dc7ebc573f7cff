# GPU box: lgx_chain (narrow tail layers in one launch): MLP / learner / rollout GPU tests, then
# bench lines alternating LGX_CHAIN=0 (one grouped launch per depth).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_chain; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_rollout.py tests/test_gpu_learner.py tests/test_gpu_learner_golden.py tests/test_gpu_distributed.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
bash tools/gpu/ab_knobs.sh "" "LGX_CHAIN=0"
