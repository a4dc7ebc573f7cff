# GPU box, round-3 closing pass: the whole -m gpu suite, smoke(), the phase clock (C2, C3), the
# default bench line (with cpu_baseline) and the rocprofv3 kernel summary of the bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_full; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
TASK=go2 N=4096 K=10 timeout -k 10 300 python tools/phase_clock.py > $O/phase_go2.txt 2>&1 || { tail -20 $O/phase_go2.txt; exit 1; }
TASK=anymal_c_rough N=4096 K=5 timeout -k 10 300 python tools/phase_clock.py > $O/phase_anymal.txt 2>&1 || { tail -20 $O/phase_anymal.txt; exit 1; }
grep "task " $O/phase_go2.txt $O/phase_anymal.txt
timeout -k 10 420 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -n 1 $O/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no_cpu_baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
tail -n 1 $O/bench_prof.json | cut -c1-300
