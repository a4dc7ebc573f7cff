# round 6: block placement probe; the persistent kernel with staggered co-resident blocks
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_stag; mkdir -p $O
cd $R
D=$R/legged_gym_custom_amd/lib/dev
timeout -k 10 60 python tools/exp/placement.py > $O/placement.log 2>&1 || { tail $O/placement.log; exit 1; }
cat $O/placement.log
for st in "0 0" "1 10000" "2 10000" "1 20000" "2 20000"; do
  set -- $st
  LGX_S8_STAGGER=$1 LGX_S8_STAGGER_DELAY=$2 PYTHONPATH=.:tools timeout -k 10 200 python -u tools/s8_clock.py $D/liblgx_s8_clock.so > $O/clock_$1_$2.log 2>&1 || { tail $O/clock_$1_$2.log; exit 1; }
  echo "== stagger $1 delay $2"; grep -E "^==" $O/clock_$1_$2.log | head -5
  LGX_S8_LIB=$D/liblgx_s8_knobs.so LGX_S8_STAGGER=$1 LGX_S8_STAGGER_DELAY=$2 PYTHONPATH=.:tests timeout -k 10 200 python tools/s8_mb_ab.py 2>$O/mb.err | tail -1 || { tail $O/mb.err; exit 1; }
done
