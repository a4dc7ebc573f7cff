# Round-5 env-kernel baseline: PMC passes (tools/gpu/pmc_env.sh) and the phase clock (Go2 4096,
# plain and crowded states). Usage: bash tools/gpu/r05_env_profile.sh <tag>
set -o pipefail
TAG=${1:-r05}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/envprof_$TAG
mkdir -p $O
cd $R
bash tools/gpu/pmc_env.sh $TAG > $O/pmc.log 2>&1 || { echo pmc failed; tail -20 $O/pmc.log; exit 1; }
timeout -k 10 300 python3 tools/phase_clock.py > $O/phase_go2.txt 2>&1 || { echo phase failed; tail $O/phase_go2.txt; exit 1; }
STATE=crowded timeout -k 10 300 python3 tools/phase_clock.py > $O/phase_go2_crowded.txt 2>&1 || exit 1
tail -25 $O/phase_go2.txt
cat $O/pmc.log | tail -30
