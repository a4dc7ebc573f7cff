# GEMM variant libraries: parity tests (test_gpu_mlp, learner) on each, then the A/B timing.
# Usage: VARIANTS="cur pf3" bash tools/gpu/exp_mlp_check.sh   (tools/exp/liblgx_mlp_<v>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in $VARIANTS; do
  echo "== tests $v"
  LGX_MLP_LIB=$PWD/tools/exp/liblgx_mlp_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py tests/test_gpu_learner.py tests/test_gpu_learner_golden.py 2>&1 | tail -2 || exit 1
done
bash tools/gpu/exp_gemm.sh
