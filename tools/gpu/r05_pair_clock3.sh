set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pair3
mkdir -p $O
cd $R
for epw in 1 2; do
  LGX_ENVS_PER_WAVE=$epw timeout -k 10 200 python -u tools/phase_clock.py > $O/clock_epw${epw}.txt 2>&1 || exit 1
done
for f in $O/clock_*.txt; do echo "== $f"; grep -A9 "^last step" $f | cut -c1-400; grep "^task" $f; done
