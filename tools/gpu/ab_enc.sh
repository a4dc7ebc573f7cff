# the act kernel with the encoders inside (LGX_ACT_ENC_IN_KERNEL=1) vs the encoders as grouped
# launches before it (default): the fused-act tests with the knob on, bench A/B alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
LGX_ACT_ENC_IN_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_s8_act.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  LGX_ACT_ENC_IN_KERNEL=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_on_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_on_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('in-kernel', b['value'], b['collection_s'], b['learn_s'])"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_off_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('grouped', b['value'], b['collection_s'], b['learn_s'])"
done
