# GPU box: straight-line GEMM K loop (counted staging waits): the MLP / learner GPU tests, then
# bench lines alternating the previous liblgx_mlp build (build/var/liblgx_mlp_old.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_pipe; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_rollout.py tests/test_gpu_learner.py tests/test_gpu_learner_golden.py tests/test_gpu_distributed.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product old product old; do
  if [ $v = product ]; then L=""; else L="LGX_MLP_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_mlp_${OLD:-old}.so"; fi
  env $L timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["roofline_learner"]["us_per_launch"])')"
done
