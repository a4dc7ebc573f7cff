# GPU box: single-buffered weight-gradient tiles at three blocks per CU (LGX_DW_SB1=1) vs the
# double-buffered product: learner / MLP GPU tests under the knob, GEMM timings, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sb1; mkdir -p $O
LGX_DW_SB1=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_learner.py tests/test_gpu_learner_golden.py -m gpu -x -q -p no:cacheprovider \
  --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in 0 1 0 1; do
  LGX_DW_SB1=$v timeout -k 10 200 python tools/gemm_variants.py > $O/gemm_$v.log 2>&1 || { tail -20 $O/gemm_$v.log; exit 1; }
  echo "sb1=$v: $(tail -n 1 $O/gemm_$v.log)"
done
for v in 0 1 0 1; do
  LGX_DW_SB1=$v timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "sb1=$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["roofline_learner"]["us_per_launch"])')"
done
