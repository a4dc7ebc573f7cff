# round-6 closing measurements: the full -m gpu suite + smoke, the default bench line (with
# cpu_baseline), env-kernel PMC (r06), rocprofv3 kernel stats of the profiled bench, the C4
# (go2_parkour, 8192 envs) and C3 (anymal_c_rough) lines. Usage: bash tools/gpu/r06_close.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $O/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_default_line.json
python -c "import json; b=json.load(open('$O/bench_default_line.json')); print('default', b['value'], b['ms_per_step'])"
[ -n "$NOPMC" ] || { bash tools/gpu/pmc_env.sh r06 > $O/pmc_env.txt 2>&1 || { tail -5 $O/pmc_env.txt; exit 1; }; tail -8 $O/pmc_env.txt; }
cd $R
bash tools/gpu/prof_kernels.sh r06 > $O/prof_head.txt 2>&1 || { tail -5 $O/prof_head.txt; exit 1; }
cp gpurun_out/prof_r06/kernel_stats.csv $O/bench_kernel_stats.csv && tail -1 gpurun_out/prof_r06/bench.json > $O/bench_profiled_line.json
head -24 $O/prof_head.txt
[ -n "$NOCX" ] && exit 0
cd $R
timeout -k 10 600 python bench.py --task go2_parkour --num_envs 8192 --no_cpu_baseline > $O/bench_c4.log 2>&1 || exit $?
tail -1 $O/bench_c4.log > $O/bench_c4_line.json
timeout -k 10 600 python bench.py --task anymal_c_rough --no_cpu_baseline > $O/bench_c3.log 2>&1 || exit $?
tail -1 $O/bench_c3.log > $O/bench_c3_line.json
for f in bench_c4_line bench_c3_line bench_profiled_line; do python -c "import json; b=json.load(open('$O/$f.json')); print('$f', b['value'], b.get('ms_per_step'))"; done
