# the act path's critic launch on a side stream (default) vs one launch (LGX_ACT_SPLIT=0): tests,
# an iteration trace, then bench A/B alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8_act.py tests/test_gpu_rollout.py tests/test_gpu_learner_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/act_tests.log 2>&1
rc=$?; tail -3 gpurun_out/act_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/prof_iter.sh > /dev/null || exit $?
head -14 gpurun_out/prof_iter/gaps.txt
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_on_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_on_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('split', b['value'], b['collection_s'], b['learn_s'])"
  LGX_ACT_SPLIT=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_off_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('one', b['value'], b['collection_s'], b['learn_s'])"
done
