# DAgger minibatch kernel: its tests, phase clocks (exp/mlp_adclk.so) and update_dagger timing fused / not.
# Usage: bash tools/gpu/dagger_check.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dagger; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "adaptation_train or dagger" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
LGX_MLP_LIB=exp/mlp_adclk.so PYTHONPATH=. timeout -k 10 120 python tools/adapt_clock.py 2>&1 | grep -v amdgpu.ids || exit 1
for f in 1 0; do
  LGX_DAGGER_FUSED=$f REPS=3 PYTHONPATH=. timeout -k 10 200 python tools/prof_dagger.py 2>&1 | grep "update_dagger" | sed "s/^/fused=$f /" || exit 1
done
