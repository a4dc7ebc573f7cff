set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2 3 4; do
  LGX_LIB=$PWD/legged_gym_custom_amd/lib/stages/liblgx_s$k.so timeout -k 10 300 python tools/kernel_timing.py > gpurun_out/kt_s$k.log 2>&1 || exit 1
  echo "stage $k: $(grep 'full step' gpurun_out/kt_s$k.log)"
done
