# Instruction-cache counters for the env-step kernel (tools/env_kernel_driver.py) and the
# loss heads (tools/heads_timing.py): one SQC counter per pass. Usage: bash tools/gpu/pmc_icache.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_icache
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/p$i -- python3 $R/tools/env_kernel_driver.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/h$i -- python3 $R/tools/heads_timing.py > $O/h$i.log 2>&1 || { echo "heads pass $i failed"; exit 1; }
done
cd $R && python3 - <<'PY'
import collections, csv, glob, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmc_icache"
for pre, match in (("p", "env_step_kernel"), ("h", "loss_heads_bwd"), ("h", "aux_loss_bwd"), ("h", "ppo_head_fwd")):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(O, pre + "*", "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if match in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(match, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
