# the encoders' input gradients as one chain launch (LGX_S8_CHAIN_DX=1) vs their grouped levels:
# S8 / update / learner tests with it on, an iteration trace with it on, bench A/B alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LGX_S8_CHAIN_DX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/chain_tests.log 2>&1
rc=$?; tail -3 gpurun_out/chain_tests.log; [ $rc -eq 0 ] || exit $rc
LGX_S8_CHAIN_DX=1 bash tools/gpu/prof_iter.sh > /dev/null || exit $?
sed -n '/---- minibatch/,/---- rollout/p' gpurun_out/prof_iter/seq.txt
cd $R
for i in 1 2; do
  LGX_S8_CHAIN_DX=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_on_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_on_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('dx chain', b['value'], b['collection_s'], b['learn_s'])"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_off_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('dx levels', b['value'], b['collection_s'], b['learn_s'])"
done
