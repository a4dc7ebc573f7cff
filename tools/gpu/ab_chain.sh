# the encoders' forward as one chain launch (default) vs their grouped levels (LGX_S8_CHAIN=0):
# S8 / update / learner tests, an iteration trace, bench A/B alternating on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_s8_act.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/chain_tests.log 2>&1
rc=$?; tail -5 gpurun_out/chain_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/prof_iter.sh > /dev/null || exit $?
head -24 gpurun_out/prof_iter/gaps.txt; head -22 gpurun_out/prof_iter/seq.txt
cd $R
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_on_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_on_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('chain', b['value'], b['collection_s'], b['learn_s'])"
  LGX_S8_CHAIN=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_off_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('levels', b['value'], b['collection_s'], b['learn_s'])"
done
