# liblgx_mlp A/B on one box: learner tests on the tree's build, then rocprofv3 kernel stats of the
# bench with the tree's liblgx_mlp.so and with exp/mlp_old.so (LGX_MLP_LIB), alternating.
# Usage: bash tools/gpu/mlp_ab.sh "<kernel name regex>"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner_golden.py tests/test_gpu_learner.py tests/test_gpu_s8_update.py 2>&1 | tail -1
for v in new old new old; do
  if [ $v = old ]; then export LGX_MLP_LIB=$R/exp/mlp_old.so; else unset LGX_MLP_LIB; fi
  echo "== $v"; bash tools/gpu/prof_bench.sh 2>&1 | grep -E "$1" || exit 1
done
