# round 5 diagnostics: teacher-forced / free-running update vs the reference probe (go2_c2),
# env-step kernel time and per-wave cycles vs waves per SIMD
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/diag1
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/env_scaling.py > $O/env_scaling.txt 2>&1 || exit 1
N=1024 timeout -k 10 200 python -u tools/phase_clock.py > $O/phase_1024.txt 2>&1 || exit 1
N=2048 timeout -k 10 200 python -u tools/phase_clock.py > $O/phase_2048.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/dbg_teacher_forced.py diag/probe_c2.npz go2_c2 > $O/tf_c2.log 2>&1 || exit 1
cat $O/env_scaling.txt; grep -A3 "task go2" $O/phase_1024.txt $O/phase_2048.txt; cat $O/tf_c2.log | grep -v Warn
