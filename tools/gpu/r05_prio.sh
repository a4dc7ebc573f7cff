# env kernel phase clock: issue-priority variants (row-count priority, wave-slot priority) x envs per wave
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prio
mkdir -p $O
cd $R
L=$R/legged_gym_custom_amd/lib
for epw in 1 2; do
  for v in prof prof_slot prof_slotonly; do
    PROF_LIB=$L/liblgx_$v.so LGX_ENVS_PER_WAVE=$epw timeout -k 10 200 python -u tools/phase_clock.py > $O/clock_${v}_epw${epw}.txt 2>&1 || exit 1
  done
done
for f in $O/clock_*.txt; do echo "== $f"; grep "^task" $f; grep "slowest 1 %" $f; done
