set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_s8clk2; mkdir -p $O
cd $R
D=$R/legged_gym_custom_amd/lib/dev
timeout -k 10 300 python -u -m pytest tests/test_gpu_s8.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PYTHONPATH=.:tools timeout -k 10 200 python -u tools/s8_clock.py $D/liblgx_s8_clock.so > $O/clock.log 2>&1 || { tail $O/clock.log; exit 1; }
grep -v "last wave" $O/clock.log
for i in 1 2; do
PYTHONPATH=.:tests timeout -k 10 200 python tools/s8_mb_ab.py > $O/mb_new.json 2>$O/mb.err || { tail $O/mb.err; exit 1; }
LGX_S8_LIB=$D/liblgx_s8_old.so PYTHONPATH=.:tests timeout -k 10 200 python tools/s8_mb_ab.py > $O/mb_old.json 2>$O/mb.err || { tail $O/mb.err; exit 1; }
cat $O/mb_new.json $O/mb_old.json
done
