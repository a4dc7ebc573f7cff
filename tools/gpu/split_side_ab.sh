# the weight split beside the encoder chain (LGX_SPLIT_SIDE): learner tests, then bench A/B, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py tests/test_gpu_graph_allreduce.py 2>&1 | tail -1
for v in 1 0 1 0; do
  LGX_SPLIT_SIDE=$v timeout -k 10 300 python bench.py --no_cpu_baseline > gpurun_out/split_side_$v.log 2>&1 || exit 1
  python -c "import json; b=json.loads(open('gpurun_out/split_side_$v.log').read().strip().splitlines()[-1]); print('side=$v', b['value'], 'learn_s', b['learn_s'])"
done
