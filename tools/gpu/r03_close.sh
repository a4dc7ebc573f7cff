# Round-3 closing pass on the product build: the full -m gpu suite, smoke, the default bench
# line (with cpu_baseline), the rocprofv3 kernel summary of the bench command, and the C3 / C4
# lines. Usage: bash tools/gpu/r03_close.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_close; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -n 2 $O/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 420 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -n 1 $O/bench_default.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no_cpu_baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
cd $R
timeout -k 10 300 python bench.py --task anymal_c_rough --num_envs 4096 --no_cpu_baseline > $O/bench_anymal_c_rough.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
tail -n 1 $O/bench_anymal_c_rough.json | cut -c1-300
timeout -k 10 300 python bench.py --task go2_parkour --num_envs 8192 --no_cpu_baseline > $O/bench_go2_parkour.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
tail -n 1 $O/bench_go2_parkour.json | cut -c1-300
