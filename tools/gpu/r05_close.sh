# round-5 closing measurements: env-kernel PMC of the paired kernel (r05b), rocprofv3 kernel stats
# of the profiled bench, the C4 (go2_parkour, 8192 envs) and C3 (anymal_c_rough) lines, and the
# DAgger iteration timing. Usage: bash tools/gpu/r05_close.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05
mkdir -p $O
cd $R
bash tools/gpu/pmc_env.sh r05b > $O/pmc_env.txt 2>&1 || { tail -5 $O/pmc_env.txt; exit 1; }
tail -8 $O/pmc_env.txt
cd $R
bash tools/gpu/prof_kernels.sh r05 > $O/prof_head.txt 2>&1 || { tail -5 $O/prof_head.txt; exit 1; }
cp gpurun_out/prof_r05/kernel_stats.csv $O/bench_kernel_stats.csv && tail -1 gpurun_out/prof_r05/bench.json > $O/bench_profiled_line.json
head -24 $O/prof_head.txt
cd $R
timeout -k 10 600 python bench.py --task go2_parkour --num_envs 8192 --no_cpu_baseline > $O/bench_c4.log 2>&1 || exit $?
tail -1 $O/bench_c4.log > $O/bench_c4_line.json
timeout -k 10 600 python bench.py --task anymal_c_rough --no_cpu_baseline > $O/bench_c3.log 2>&1 || exit $?
tail -1 $O/bench_c3.log > $O/bench_c3_line.json
for f in bench_c4_line bench_c3_line bench_profiled_line; do python -c "import json; b=json.load(open('$O/$f.json')); print('$f', b['value'], b.get('ms_per_step'), b.get('env_kernel'))"; done
timeout -k 10 300 python tools/dagger_timing.py > $O/dagger_timing.txt 2>&1 || exit $?
tail -3 $O/dagger_timing.txt
