# GPU box: the weight-gradient group's block budget (LGX_DW_SLOTS -> split-K), dWgroup timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_slots; mkdir -p $O
for sl in 512 384 448 640 512 384 448 640; do
  LGX_DW_SLOTS=$sl timeout -k 10 200 python tools/gemm_variants.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
  echo "slots=$sl: $(tail -n 1 $O/gemm.log | grep -o 'dWgroup.*')"
done
