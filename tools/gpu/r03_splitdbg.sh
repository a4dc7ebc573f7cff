set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_split; mkdir -p $O
LGX_DW_SLOTS=512 timeout -k 10 300 python tools/dbg_split_update.py $O/s6.npz > $O/s6.log 2>&1 || { tail -20 $O/s6.log; exit 1; }
LGX_DW_SLOTS=768 timeout -k 10 300 python tools/dbg_split_update.py $O/s9.npz > $O/s9.log 2>&1 || { tail -20 $O/s9.log; exit 1; }
python tools/dbg_split_update.py --compare $O/s6.npz $O/s9.npz
rm -f $O/*.npz
