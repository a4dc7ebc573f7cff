# GPU box: env kernel with LDS-only block barriers (no wait on outstanding global stores):
# env GPU parity on that build, then C2 / C3 / C4 bench lines alternating it with the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_ldssync; mkdir -p $O
LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_ldssync.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trajectory.py tests/test_gpu_terrain.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product ldssync product ldssync; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --no_cpu_baseline > $O/c2_$v.log 2>&1 || { tail -20 $O/c2_$v.log; exit 1; }
  echo "c2 $v: $(tail -n 1 $O/c2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/c3_$v.log 2>&1 || { tail -20 $O/c3_$v.log; exit 1; }
  echo "c3 $v: $(tail -n 1 $O/c3_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
for v in product ldssync; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
  echo "c4 $v: $(tail -n 1 $O/c4_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
