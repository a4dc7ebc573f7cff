set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --task go2_parkour --num_envs 8192 --steps 5 --warmup 2 --no_cpu_baseline > gpurun_out/bench_parkour.log 2>&1
rc=$?
echo "parkour rc=$rc"; tail -3 gpurun_out/bench_parkour.log
exit $rc
