# round 6, first GPU pass: the tests touched this round, then the default bench line and its
# rocprofv3 kernel stats (the A/B baseline of this round's box)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06a; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_distributed_bench.py \
  "tests/test_gpu_learner_golden.py::test_gpu_adam_moments_after_update" -m gpu -v -s -p no:cacheprovider -rf \
  --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_line.json
bash tools/gpu/prof_kernels.sh r06a > $O/prof_head.txt 2>&1 || { cat $O/prof_head.txt; exit 1; }
cp gpurun_out/prof_r06a/kernel_stats.csv $O/kernel_stats.csv
head -25 $O/prof_head.txt
python -c "import json; b=json.load(open('$O/bench_line.json')); print(b['value'], b['ms_per_step'], b['collection_s'], b['learn_s'], b['env_kernel'], b['paths'], b['binaries'])"
