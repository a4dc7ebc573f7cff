set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_sb1; mkdir -p $O
for v in 0 1; do
  LGX_DW_SB1=$v timeout -k 10 200 python tools/check_dw_group.py > $O/chk_$v.log 2>&1 || { tail -20 $O/chk_$v.log; exit 1; }
  echo "sb1=$v"; cat $O/chk_$v.log | grep -v amdgpu.ids
done
