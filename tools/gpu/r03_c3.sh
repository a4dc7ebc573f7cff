# GPU box (round 3): ANYmal parity tests on the product build, then the C3 rollout bench on the
# product (SEA variant at 2 waves/SIMD) and the 3- / 4-wave builds, then the hipBLASLt A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_c3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_terrain.py tests/test_gpu_parity.py tests/test_gpu_mlp.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "anymal or golden or empty_input" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in product w3 w4; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
timeout -k 10 300 python tools/ab_blaslt.py --json $O/ab_blaslt.json > $O/ab_blaslt.log 2>&1 || { tail -20 $O/ab_blaslt.log; exit 1; }
tail -3 $O/ab_blaslt.log
