# GPU box: learner GEMMs with 8-wave 128x128 blocks (LGX_MLP_NW=8) — parity tests under the knob,
# then bench lines alternating the 4-wave product and the 8-wave variants (2 rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_nw; mkdir -p $O
LGX_MLP_NW=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_learner_golden.py tests/test_gpu_learner.py -m gpu -x -q -p no:cacheprovider -k "not single_launches_bitwise" \
  --timeout 200 --timeout-method thread > $O/pytest_nw8.log 2>&1 || { tail -30 $O/pytest_nw8.log; exit 1; }
tail -1 $O/pytest_nw8.log
for r in 1 2; do
  for v in "" "LGX_MLP_NW=8" "LGX_MLP_NW_DW=8" "LGX_MLP_NW=8 LGX_MLP_NW_DW=4"; do
    env $v timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    echo "[$v] $(tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["roofline_learner"]["us_per_launch"])')"
  done
done
