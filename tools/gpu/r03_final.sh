# Round-3 measurement pass: default bench line, the rocprofv3 kernel summary of the profiled
# bench command, and env-kernel PMC (instruction mix, waits, HBM traffic) for Go2 (C2),
# anymal_c_rough (C3) and go2_parkour (C4). Usage: bash tools/gpu/r03_final.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_final; mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no_cpu_baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
cd $R
TASK=go2 N=4096 timeout -k 10 400 bash tools/gpu/pmc_env.sh r03 > $O/pmc_go2.log 2>&1 || { tail -20 $O/pmc_go2.log; exit 1; }
TASK=anymal_c_rough N=4096 timeout -k 10 400 bash tools/gpu/pmc_env.sh r03 > $O/pmc_c3.log 2>&1 || { tail -20 $O/pmc_c3.log; exit 1; }
TASK=go2_parkour N=8192 timeout -k 10 400 bash tools/gpu/pmc_env.sh r03 > $O/pmc_c4.log 2>&1 || { tail -20 $O/pmc_c4.log; exit 1; }
cp $R/gpurun_out/pmc_env_r03_*/r03_*.txt $R/gpurun_out/pmc_env_r03_*/r03_*.json $O/
tail -5 $O/pmc_go2.log $O/pmc_c3.log $O/pmc_c4.log
