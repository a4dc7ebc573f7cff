set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_rollout.py -x -q -p no:cacheprovider > gpurun_out/pytest_parity.log 2>&1 && echo PARITY_OK || { tail -20 gpurun_out/pytest_parity.log; exit 1; }
for n in 1792 2816 4096 8192; do
  N=$n timeout -k 10 300 python tools/kernel_timing.py > gpurun_out/kt_$n.log 2>&1 || exit 1
  echo "N=$n: $(grep 'full step' gpurun_out/kt_$n.log) | $(grep 'iterations=0' gpurun_out/kt_$n.log)"
done
