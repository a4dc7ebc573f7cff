# A/B of env-kernel phase-clock builds (alternating runs): bash tools/gpu/ab_env.sh <variant lib>...
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in liblgx_prof.so "$@"; do
    echo "== $v"
    PROF_LIB=$PWD/legged_gym_custom_amd/lib/$v K=30 timeout -k 10 200 python tools/phase_clock.py > gpurun_out/ab_$v.$r.txt 2>&1 || exit 1
    grep -E "^task|^pgs|^kinematics|^dynamics" gpurun_out/ab_$v.$r.txt
  done
done
