# GPU box: SEA-variant spill fix (k-outer cell step, per-pass opaque weight table): ANYmal parity
# tests, C3 rollout bench for the product / the hoisted-weights build / the gate-row build, then
# the C3 env-kernel PMC (traffic) of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sea2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_terrain.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "anymal or sea or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product sea_hoist sea_rows product; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
TASK=anymal_c_rough N=4096 timeout -k 10 400 bash tools/gpu/pmc_env.sh r03b > $O/pmc_c3.log 2>&1 || { tail -20 $O/pmc_c3.log; exit 1; }
grep -E "wait fraction|instructions per" $O/pmc_c3.log
grep traffic_bytes $O/pmc_c3.log
