set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/diag1
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/dbg_teacher_forced.py diag/probe_c2.npz go2_c2 > $O/tf_c2.log 2>&1 || { tail -20 $O/tf_c2.log; exit 1; }
grep -v Warn $O/tf_c2.log
