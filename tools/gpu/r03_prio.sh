# GPU box: wave issue priority by constraint-system size (-DLGX_ROW_PRIO=t: priority 1/2/3 above
# t / 2t / 3t rows) vs the product: C2, C3, C4 bench lines (env-kernel HIP-event averages).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_prio; mkdir -p $O
for v in product prio12 prio15 prio0 product prio12 prio15 prio0; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --no_cpu_baseline > $O/c2_$v.log 2>&1 || { tail -20 $O/c2_$v.log; exit 1; }
  echo "c2 $v: $(tail -n 1 $O/c2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
for v in product prio12 prio15 prio0; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --steps 10 --warmup 2 --no_cpu_baseline > $O/c3_$v.log 2>&1 || { tail -20 $O/c3_$v.log; exit 1; }
  echo "c3 $v: $(tail -n 1 $O/c3_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
  env $L timeout -k 10 300 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > $O/c4_$v.log 2>&1 || { tail -20 $O/c4_$v.log; exit 1; }
  echo "c4 $v: $(tail -n 1 $O/c4_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"])')"
done
