# round 6: the heads-tail launch with its PPO head rows spread over (row, action) threads — tests, then
# per-level minibatch traces against the previous build (lib/dev/liblgx_mlp_old.so), twice on one box
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_heads}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py tests/test_gpu_mlp.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in new old new2 old2; do
  L=""; [ "${v#old}" != "$v" ] && L=$R/legged_gym_custom_amd/lib/dev/liblgx_mlp_old.so
  LGX_MLP_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 $R/tools/s8_mb_ab.py > $O/mb_$v.json 2> $O/mb_$v.err || { tail $O/mb_$v.err; exit 1; }
  echo "$v $(cat $O/mb_$v.json)"
done
cd $R && python3 tools/trace_levels.py $O/tr_new/run_kernel_trace.csv $O/tr_old/run_kernel_trace.csv $O/tr_new2/run_kernel_trace.csv $O/tr_old2/run_kernel_trace.csv
