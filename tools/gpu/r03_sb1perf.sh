# GPU box: weight-gradient group timing, single-buffered 3-blocks-per-CU tiles (LGX_DW_SB1=1)
# with their own split (9) and with the product's (6), vs the product kernel; then bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sb1; mkdir -p $O
for cfg in "LGX_DW_SB1=0" "LGX_DW_SB1=1" "LGX_DW_SB1=1 LGX_DW_SLOTS=512" "LGX_DW_SB1=0 LGX_DW_SLOTS=768"; do
  env $cfg timeout -k 10 200 python tools/gemm_variants.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
  echo "$cfg: $(tail -n 1 $O/gemm.log | grep -o 'dWgroup.*')"
  env $cfg timeout -k 10 200 python tools/dw_cache_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
  echo "   probe: $(tail -n 1 $O/probe.log)"
done
for cfg in "LGX_DW_SB1=0" "LGX_DW_SB1=1" "LGX_DW_SB1=0" "LGX_DW_SB1=1"; do
  env $cfg timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  echo "$cfg: $(tail -n 1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["roofline_learner"]["us_per_launch"])')"
done
