# GPU box: terrain-contact parity (the wave-distributed query) and C3 / C4 timing against the
# one-candidate-per-lane build.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_terr; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_terrain.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in product terr_lane; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/c3_$v.log 2>&1 || { tail -20 $O/c3_$v.log; exit 1; }
  echo "C3 $v: $(tail -1 $O/c3_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
  env $L timeout -k 10 300 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
  echo "C4 $v: $(tail -1 $O/c4_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
