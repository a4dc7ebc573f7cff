# bench A/B: the one-launch act path vs the grouped launches (LGX_FUSED_ACT=0), alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_on_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_on_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('fused', b['value'], b['collection_s'], b['learn_s'])"
  LGX_FUSED_ACT=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_off_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); print('grouped', b['value'], b['collection_s'], b['learn_s'])"
done
