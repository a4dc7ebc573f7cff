# A/B of liblgx_mlp.so builds: the learner/MLP GPU tests on the product build, then the bench
# line alternating product and each variant (tools/exp/liblgx_mlp_<v>.so), then kernel-trace
# stats of 1 runner iteration per build (KSEL: kernel-name filter).
# bash tools/gpu/ab_mlp.sh <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$PWD; O=$R/gpurun_out/ab_mlp; rm -rf $O; mkdir -p $O
# a variant "env:NAME=value" runs the product build with that environment variable set
lib_of() { case $1 in product|env:*) echo $R/legged_gym_custom_amd/lib/liblgx_mlp.so;; *) echo $R/tools/exp/liblgx_mlp_$1.so;; esac; }
env_of() { case $1 in env:*) echo ${1#env:};; *) echo LGX_AB_NONE=1;; esac; }
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-learner or mlp or rollout or train}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2; do
  for v in product "$@"; do
    env $(env_of $v) LGX_MLP_LIB=$(lib_of $v) timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no_cpu_baseline > $O/b_${v//[:=]/_}_$r.log 2>&1 || { tail -5 $O/b_${v//[:=]/_}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v//[:=]/_}_$r.log').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['ms_per_step'], d['collection_s'], d['learn_s'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in product "$@"; do
  export $(env_of $v); LGX_MLP_LIB=$(lib_of $v) K=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v//[:=]/_} -- python3 $R/tools/prof_iter.py > $O/prof_${v//[:=]/_}.log 2>&1 || exit 1
  f=$(find $O/prof_${v//[:=]/_} -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in '${KSEL:-tail splitk loss_heads gemm_group}'.split()): print('  ', r['Name'].split('(')[0][-44:], r['Calls'], r['AverageNs'])
"
  find $O/prof_${v//[:=]/_} -name "*_kernel_trace.csv" -delete
  unset $(env_of $v | cut -d= -f1)
done
