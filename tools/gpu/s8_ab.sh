# S8 library A/B on one box: the learner tests on the tree's build, then rocprofv3 kernel stats of the
# bench with the tree's liblgx_s8.so and with exp/s8_old.so (LGX_S8_LIB), alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py 2>&1 | tail -1
for v in new old new old; do
  if [ $v = old ]; then export LGX_S8_LIB=$R/exp/s8_old.so; else unset LGX_S8_LIB; fi
  echo "== $v"; bash tools/gpu/prof_bench.sh 2>&1 | grep -E "s8_gemm_kernel|chain_kernel<2" || exit 1
done
