# phase clock, one vs two envs per wave (Go2 plane)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pair
mkdir -p $O
cd $R
for n in 1024 4096; do
  for epw in 1 2; do
    LGX_ENVS_PER_WAVE=$epw N=$n timeout -k 10 200 python -u tools/phase_clock.py > $O/clock_n${n}_epw${epw}.txt 2>&1 || exit 1
  done
done
for f in $O/clock_n*_epw*.txt; do echo "== $f"; grep -A18 "^task" $f; done
