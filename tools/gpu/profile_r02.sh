# Round profile on the GPU box (r02): rocprofv3 kernel-trace stats of the bench command and
# its JSON line, the default bench line (with cpu_baseline), the go2_parkour 8192-env bench
# line, and kernel-trace stats of the C3/C4 env kernels. Outputs in gpurun_out/prof_r02/.
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 $R/bench.py --steps 10 --warmup 2 --no_cpu_baseline --kernel_iters 20 > $O/bench.log 2>&1 || exit $?
TASK=go2_parkour N=8192 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/parkour -- python3 $R/tools/env_kernel_driver.py > $O/parkour.log 2>&1 || exit $?
TASK=anymal_c_rough N=4096 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/anymal -- python3 $R/tools/env_kernel_driver.py > $O/anymal.log 2>&1 || exit $?
find $O -name "*_kernel_trace.csv" -delete
cd $R
timeout -k 10 600 python bench.py > $O/default.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > $O/parkour_bench.log 2>&1 || exit $?
mkdir -p $O/profiles
cp $(find $O/trace -name "*_kernel_stats.csv") $O/profiles/${TAG}_bench_kernel_stats.csv
cp $(find $O/parkour -name "*_kernel_stats.csv") $O/profiles/${TAG}_env_parkour_n8192_kernel_stats.csv
cp $(find $O/anymal -name "*_kernel_stats.csv") $O/profiles/${TAG}_env_anymal_rough_n4096_kernel_stats.csv
grep '"metric"' $O/bench.log | tail -1 > $O/profiles/${TAG}_bench_line.json
grep '"metric"' $O/default.log | tail -1 > $O/profiles/${TAG}_bench_default_line.json
grep '"metric"' $O/parkour_bench.log | tail -1 > $O/profiles/${TAG}_bench_parkour_n8192_line.json
ls $O/profiles; cut -c1-400 $O/profiles/${TAG}_bench_default_line.json
