# round 6: the weight-gradient group's split-K residency target (LGX_S8_DW_SLOTS on a -DLGX_DEV_KNOBS build)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_dwslots}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K=$R/legged_gym_custom_amd/lib/dev/liblgx_s8_knobs.so
for v in 512 384 768 1024 512 384 768 1024; do
  LGX_S8_LIB=$K LGX_S8_DW_SLOTS=$v PYTHONPATH=$R:$R/tests timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_${v}_$RANDOM -o run -- python3 $R/tools/s8_mb_ab.py > $O/mb_$v.json 2> $O/mb_$v.err || { tail $O/mb_$v.err; exit 1; }
  echo "slots $v $(cat $O/mb_$v.json)"
done
