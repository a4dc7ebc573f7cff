set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sb1; mkdir -p $O
for cfg in "LGX_DW_SB1=0" "LGX_DW_SB1=1" "LGX_DW_SB1=1 LGX_DW_SLOTS=512" "LGX_DW_SB1=0 LGX_DW_SLOTS=768"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_learner_golden.py -m gpu -q -p no:cacheprovider -s \
    --timeout 150 --timeout-method thread -k "moments or mb0 or minibatch0" > $O/dbg.log 2>&1
  echo "== $cfg: rc=$?"; grep -E "Adam moments|moved the other way|AssertionError: \(|passed|failed" $O/dbg.log | head -12
done
