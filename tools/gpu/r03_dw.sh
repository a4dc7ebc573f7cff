# GPU box: the wide weight-gradient kernel (8 waves, 128 x 256 tiles): learner GPU tests, the
# GEMM variant timings (product PF 3 / PF 2 build / the 4-wave kernel via LGX_DW_WIDE=0), the
# dW cache-state probe, then bench lines alternating wide and 4-wave.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_dw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_learner.py tests/test_gpu_learner_golden.py -m gpu -x -q -p no:cacheprovider \
  --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in product pf2 narrow; do
  case $v in product) L="";; pf2) L="LGX_MLP_LIB=$GRAFT_REPO_ROOT/build/var/liblgx_mlp_pf2.so";; narrow) L="LGX_DW_WIDE=0";; esac
  env $L timeout -k 10 200 python tools/gemm_variants.py > $O/gemm_$v.log 2>&1 || { tail -20 $O/gemm_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/gemm_$v.log)"
  env $L timeout -k 10 200 python tools/dw_cache_probe.py > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
  echo "$v probe: $(tail -n 1 $O/probe_$v.log)"
done
for v in product narrow product narrow; do
  case $v in product) L="";; narrow) L="LGX_DW_WIDE=0";; esac
  env $L timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["roofline_learner"]["us_per_launch"])')"
done
