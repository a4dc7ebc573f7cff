# round 6: per-block cycle accounts of the persistent kernel vs the per-tile kernel, and an
# in-process kernel trace of the update's minibatches with each library
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_s8clk; mkdir -p $O
cd $R
D=$R/legged_gym_custom_amd/lib/dev
PYTHONPATH=.:tools timeout -k 10 200 python -u tools/s8_clock.py $D/liblgx_s8_clock.so $D/liblgx_s8_oldclock.so > $O/clock.log 2>&1 || { tail $O/clock.log; exit 1; }
grep -v "last wave" $O/clock.log
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  L=""; [ $v = old ] && L=$D/liblgx_s8_old.so
  LGX_S8_LIB=$L PYTHONPATH=$R:$R/tests timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 $R/tools/s8_mb_ab.py > $O/mb_$v.json 2> $O/mb_$v.err || { tail $O/mb_$v.err; exit 1; }
  cat $O/mb_$v.json
done
find $O -name "*kernel_trace.csv" | head
