# phase clock at 4096: one / two envs per wave, with and without the row-count wave priority
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pair2
mkdir -p $O
cd $R
for epw in 1 2; do
  LGX_ENVS_PER_WAVE=$epw timeout -k 10 200 python -u tools/phase_clock.py > $O/clock_epw${epw}.txt 2>&1 || exit 1
  PROF_LIB=$R/legged_gym_custom_amd/lib/liblgx_prof_np.so LGX_ENVS_PER_WAVE=$epw timeout -k 10 200 python -u tools/phase_clock.py > $O/clock_epw${epw}_noprio.txt 2>&1 || exit 1
done
for f in $O/clock_*.txt; do echo "== $f"; sed -n 3,14p $f | cut -c1-60; grep "^task" $f; done
