set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_fwdreg}; mkdir -p $O
cd $R
D=$R/legged_gym_custom_amd/lib/dev
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in new old new2 old2; do
  L=""; [ "${v#old}" != "$v" ] && L=$D/liblgx_s8_old.so
  LGX_S8_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 $R/tools/s8_mb_ab.py > $O/mb_$v.json 2> $O/mb_$v.err || { tail $O/mb_$v.err; exit 1; }
  cat $O/mb_$v.json
done
