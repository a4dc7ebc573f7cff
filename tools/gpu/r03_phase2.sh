set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_phase2; mkdir -p $O
TASK=anymal_c_rough N=4096 K=5 timeout -k 10 300 python tools/phase_clock.py > $O/anymal.txt 2>&1 || { tail -20 $O/anymal.txt; exit 1; }
TASK=go2_parkour N=8192 K=5 timeout -k 10 300 python tools/phase_clock.py > $O/parkour.txt 2>&1 || { tail -20 $O/parkour.txt; exit 1; }
tail -20 $O/anymal.txt; tail -20 $O/parkour.txt
