# round 6: elements per block of the tail's per-range Adam launch (LGX_TAIL_ELEMS 1024 product vs 512 / 2048 / 4096 builds)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/legged_gym_custom_amd/lib/dev
for L in "" $D/liblgx_mlp_te512.so $D/liblgx_mlp_te2048.so $D/liblgx_mlp_te4096.so "" $D/liblgx_mlp_te512.so $D/liblgx_mlp_te2048.so $D/liblgx_mlp_te4096.so; do
  LGX_MLP_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 python tools/tail_ab.py 2>&1 | tail -1 || exit 1
done
