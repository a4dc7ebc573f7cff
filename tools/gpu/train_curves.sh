# end-to-end learning curves on the current build: go2 (1500 iterations) and go2_parkour (600)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/curves; mkdir -p $O
cd $R
ITERS=1500 timeout -k 10 500 python -u tools/train_curve.py > $O/go2.txt 2>&1 || { tail -5 $O/go2.txt; exit 1; }
tail -4 $O/go2.txt
TASK=go2_parkour ITERS=600 timeout -k 10 400 python -u tools/train_curve.py > $O/parkour.txt 2>&1 || { tail -5 $O/parkour.txt; exit 1; }
tail -4 $O/parkour.txt
