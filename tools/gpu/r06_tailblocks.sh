# round 6: tail_norms' grid (LGX_TAIL_BLOCKS 128 product vs 256 / 512 builds): lgx_ppo_tail alone (tools/tail_ab.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for L in "" $R/legged_gym_custom_amd/lib/dev/liblgx_mlp_tb256.so $R/legged_gym_custom_amd/lib/dev/liblgx_mlp_tb512.so "" $R/legged_gym_custom_amd/lib/dev/liblgx_mlp_tb256.so $R/legged_gym_custom_amd/lib/dev/liblgx_mlp_tb512.so; do
  LGX_MLP_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 python tools/tail_ab.py 2>&1 | tail -1 || exit 1
done
