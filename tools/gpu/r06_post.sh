# round 6: the tail S8 copies (isolated tail timing, product vs no-emission build) and the fused
# post-step launch (rollout tests, then the bench with LGX_POST_STEP=1/0 interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_post}; mkdir -p $O
cd $R
bash tools/gpu/r06_tail_ab.sh > $O/tail_ab.log 2>&1 || { tail -20 $O/tail_ab.log; exit 1; }
cat $O/tail_ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_mlp.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  LGX_POST_STEP=$v timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  python -c "import json; b=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('post_step=$v', b['value'], b['ms_per_step'], b['learn_s'], b['collection_s'])"
done
