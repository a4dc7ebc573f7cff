# GPU box: where the C3 SEA time goes: the product (MFMA form) vs no state round trip vs no
# actuator net at all (timing-only builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_seaexp; mkdir -p $O
for v in product sea_nostate sea_none product; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
