# GPU box: C3 bench for the SEA pair-form variants vs the product, then the GEMM bottleneck
# experiment (liblgx_mlp built without global loads / MFMAs / staging stores in the K loop).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sea3; mkdir -p $O
for v in product sea_pairs1 sea_pairs2 product; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
for v in product noload nomfma nostore mfmaonly loadonly; do
  if [ $v = product ]; then L=""; else L="LGX_MLP_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_mlp_$v.so"; fi
  env $L timeout -k 10 200 python tools/gemm_variants.py > $O/gemm_$v.log 2>&1 || { tail -20 $O/gemm_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/gemm_$v.log)"
done
