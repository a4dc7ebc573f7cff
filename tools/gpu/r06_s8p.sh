# round 6: the persistent FWD / DX kernel — S8 GEMM + update tests, then timings against the
# per-tile kernel (lib/dev/liblgx_s8_old.so = the same source with -DLGX_S8_PERSIST_DEFAULT=0)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_s8p; mkdir -p $O
cd $R
OLD=$R/legged_gym_custom_amd/lib/dev/liblgx_s8_old.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py ${EXTRA_TESTS} -m gpu -v -p no:cacheprovider -rf \
  -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "FAIL|ERROR|passed|failed" $O/tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=.:tools timeout -k 10 300 python tools/s8_one.py $OLD > $O/one.json 2> $O/one.err || { tail $O/one.err; exit 1; }
cat $O/one.json
for i in 1 2; do
  PYTHONPATH=.:tests timeout -k 10 200 python tools/s8_mb_ab.py > $O/mb_new_$i.json 2>$O/mb.err || { tail $O/mb.err; exit 1; }
  LGX_S8_LIB=$OLD PYTHONPATH=.:tests timeout -k 10 200 python tools/s8_mb_ab.py > $O/mb_old_$i.json 2>$O/mb.err || { tail $O/mb.err; exit 1; }
  cat $O/mb_new_$i.json $O/mb_old_$i.json
done
