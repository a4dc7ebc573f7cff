# A/B of env-var knobs on the bench line (alternating, 2 rounds):
#   bash tools/gpu/ab_knobs.sh "" "LGX_DW_SLOTS=640" ...   ("" = product defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_knobs; mkdir -p $O
i=0
for r in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python bench.py --no_cpu_baseline > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
    echo "[$v] $(tail -n 1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["collection_s"], d["learn_s"], d["env_kernel"]["avg_us"], d["roofline_learner"]["us_per_launch"])')"
  done
done
