# Round profile on the GPU box: kernel-trace stats of the bench command, and the env-step
# kernel's HBM traffic from two separate PMC passes. Usage: bash tools/profile_round.sh r01
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 $R/bench.py --steps 5 --warmup 3 --no_cpu_baseline --kernel_iters 20 > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -- python3 $R/tools/env_kernel_driver.py > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -- python3 $R/tools/env_kernel_driver.py > $O/write.log 2>&1
[ $? -eq 0 ] && \
TASK=go2_parkour N=8192 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/parkour -- python3 $R/tools/env_kernel_driver.py > $O/parkour.log 2>&1 && \
TASK=anymal_c_rough N=4096 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/anymal -- python3 $R/tools/env_kernel_driver.py > $O/anymal.log 2>&1
rc=$?
find $O -name "*_kernel_trace.csv" -delete
python3 $R/tools/summarize_profiles.py $O $O/profiles $TAG
tail -1 $O/bench.log
exit $rc
