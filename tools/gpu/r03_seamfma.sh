# GPU box: SEA LSTM on exact-f32 MFMA. ANYmal / SEA parity tests, then the C3 rollout bench
# alternating the product and the lane-parallel build (-DLGX_SEA_LANES), then the C3 phase clock.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_seamfma; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_terrain.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "anymal or sea or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product sea_lanes product sea_lanes; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
