set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in MFMA1 NOSPLIT BOTH; do
  echo "== $v"
  LGX_MLP_LIB=$PWD/exp/liblgx_mlp_$v.so timeout -k 10 120 python tools/bench_mlp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
