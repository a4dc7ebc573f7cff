# round 6: the S8 GEMMs with a 64-deep K step (-DLGX_S8_BK=64: 128 KB of LDS stages, one block per CU) vs the product
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_bk64}; mkdir -p $O
cd $R
V=$R/legged_gym_custom_amd/lib/dev/liblgx_s8_bk64.so
LGX_S8_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in "" $V "" $V; do
  LGX_S8_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 python3 tools/s8_mb_ab.py 2>&1 | tail -1 || exit 1
done
