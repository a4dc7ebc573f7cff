# round 6: the LDS-staged adaptation forward — its tests, then timing against the global-operand kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_adapt}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_rollout.py tests/test_gpu_learner.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
K=$R/legged_gym_custom_amd/lib/dev/liblgx_mlp_knobs.so
for v in 1 0 1 0; do
  LGX_MLP_LIB=$K LGX_ADAPT_FWD2=$v timeout -k 10 120 python tools/adapt_fwd_timing.py 2>&1 | tail -1 || exit 1
done
timeout -k 10 120 python tools/adapt_fwd_timing.py 2>&1 | tail -1
