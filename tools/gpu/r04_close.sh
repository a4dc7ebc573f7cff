# round-4 closing measurements: the default bench line (with cpu_baseline), its rocprofv3 kernel
# stats, the C4 (go2_parkour, 8192 envs) and C3 (anymal_c_rough) lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log > $O/bench_default_line.json
bash tools/gpu/prof_kernels.sh r04 > $O/prof_head.txt 2>&1 || exit $?
cp gpurun_out/prof_r04/kernel_stats.csv $O/bench_kernel_stats.csv && tail -1 gpurun_out/prof_r04/bench.json > $O/bench_profiled_line.json
cd $R
timeout -k 10 600 python bench.py --task go2_parkour --num_envs 8192 --no_cpu_baseline > $O/bench_c4.log 2>&1 || exit $?
tail -1 $O/bench_c4.log > $O/bench_c4_line.json
timeout -k 10 600 python bench.py --task anymal_c_rough --no_cpu_baseline > $O/bench_c3.log 2>&1 || exit $?
tail -1 $O/bench_c3.log > $O/bench_c3_line.json
head -25 $O/prof_head.txt
for f in bench_default_line bench_c4_line bench_c3_line; do python -c "import json; b=json.load(open('$O/$f.json')); print('$f', b['value'], b.get('ms_per_step'))"; done
