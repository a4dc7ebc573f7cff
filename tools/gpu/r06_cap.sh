set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_cap; mkdir -p $O
cd $R
D=$R/legged_gym_custom_amd/lib/dev
cd /tmp && export TMPDIR=/tmp
for v in cap4096 cap64 old; do
  L=$D/liblgx_s8_knobs.so; C=64
  [ $v = cap4096 ] && C=4096
  [ $v = old ] && L=$D/liblgx_s8_old.so
  LGX_S8_PERSIST_CAP=$C LGX_S8_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 $R/tools/s8_mb_ab.py > $O/mb_$v.json 2> $O/mb_$v.err || { tail $O/mb_$v.err; exit 1; }
  cat $O/mb_$v.json
done
