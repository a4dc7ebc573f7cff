# round 6: the weight split folded into the optimizer tail — learner tests, then the bench with
# and without it (LGX_TAIL_S8=0: the per-minibatch split launch), interleaved. Usage: bash tools/gpu/r06_tail.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_tail}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_s8_update.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py tests/test_gpu_s8.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0; do
  LGX_TAIL_S8=$v timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  python -c "import json; b=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]); print('tail_s8=$v', b['value'], b['ms_per_step'], b['learn_s'], b['collection_s'])"
done
