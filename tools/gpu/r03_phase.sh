# GPU box: per-phase cycle clock of the env kernel (dev build liblgx_prof.so) for ANYmal rough (C3)
# and Go2 flat (C2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_phase; mkdir -p $O
TASK=anymal_c_rough N=4096 K=5 timeout -k 10 300 python tools/phase_clock.py > $O/anymal.txt 2>&1 || { tail -20 $O/anymal.txt; exit 1; }
TASK=go2 N=4096 K=10 timeout -k 10 300 python tools/phase_clock.py > $O/go2.txt 2>&1 || { tail -20 $O/go2.txt; exit 1; }
tail -22 $O/anymal.txt; tail -22 $O/go2.txt
