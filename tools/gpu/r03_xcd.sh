# GPU box: XCD-aware env-to-block order. Env GPU parity tests, then bench lines (C2 go2, C4
# go2_parkour) alternating the product and the linear-order build, then the C2 env-kernel PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_xcd; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trajectory.py tests/test_gpu_terrain.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product linear product linear; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
for v in product linear; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > $O/parkour_$v.log 2>&1 || { tail -20 $O/parkour_$v.log; exit 1; }
  echo "parkour $v: $(tail -n 1 $O/parkour_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
TASK=go2 N=4096 timeout -k 10 400 bash tools/gpu/pmc_env.sh r03c > $O/pmc_go2.log 2>&1 || { tail -20 $O/pmc_go2.log; exit 1; }
grep -E "wait fraction|fetch_bytes|write_bytes|traffic_bytes" $O/pmc_go2.log
