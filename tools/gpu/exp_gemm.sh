# A/B of GEMM variant libraries (tools/gemm_variants.py), alternating, one process each.
# Usage: VARIANTS="noguard ..." bash tools/gpu/exp_gemm.sh   (tools/exp/liblgx_mlp_<v>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  LGX_MLP_LIB= timeout -k 10 120 python tools/gemm_variants.py 2>&1 | grep -v amdgpu.ids || exit 1
  for v in $VARIANTS; do
    LGX_MLP_LIB=$PWD/tools/exp/liblgx_mlp_$v.so timeout -k 10 120 python tools/gemm_variants.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
