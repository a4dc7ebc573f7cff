# Constraint-solve paths check: the GPU parity tests (incl. crowded contacts), then the
# per-step slowest-wave table of the phase-clock build on the bench workload, on crowded
# (base on the ground) and on tilted (base edge on the ground) states.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trajectory.py -x -q --timeout 120 --timeout-method thread > $O/pgs_tests.log 2>&1
rc=$?; tail -2 $O/pgs_tests.log; [ $rc -eq 0 ] || exit $rc
K=30 timeout -k 10 300 python tools/phase_clock.py > $O/phase_clock.txt 2>&1 || exit $?
STATE=crowded K=10 timeout -k 10 300 python tools/phase_clock.py > $O/phase_clock_crowded.txt 2>&1 || exit $?
STATE=tilted K=10 timeout -k 10 300 python tools/phase_clock.py > $O/phase_clock_tilted.txt 2>&1 || exit $?
for f in phase_clock phase_clock_crowded phase_clock_tilted; do grep -E "^constraint|^task" $O/$f.txt; done
