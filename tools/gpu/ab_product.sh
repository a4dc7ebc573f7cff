# A/B of product builds of liblgx.so (env-kernel time at 4096 envs, alternating runs):
# bash tools/gpu/ab_product.sh <lib name in legged_gym_custom_amd/lib>...
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in liblgx.so "$@"; do
    echo "== $v"
    LGX_LIB=$PWD/legged_gym_custom_amd/lib/$v NS=4096 K=200 timeout -k 10 200 python tools/env_scaling.py || exit 1
  done
done
