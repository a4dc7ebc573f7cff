# GPU box: SEA weights staged in the LDS arena (product) vs read from the params (gw) vs the
# fast-transcendental dev build (fast): ANYmal parity tests on product and fast, C3 bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sealds; mkdir -p $O
K="anymal or sea or actuator"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_fast.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $O/pytest_fast.log 2>&1; echo "fast build tests: $(tail -n 1 $O/pytest_fast.log)"
for r in 1 2; do for v in product gw fast; do
  if [ $v = product ]; then L=""; else L="LGX_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_$v.so"; fi
  env $L timeout -k 10 240 python bench.py --task anymal_c_rough --no_cpu_baseline > $O/bench_$v.$r.log 2>&1 || { tail -20 $O/bench_$v.$r.log; exit 1; }
  echo "$v: $(tail -1 $O/bench_$v.$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["env_kernel"]["avg_us"])')"
done; done
