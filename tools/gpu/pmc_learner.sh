# PMC passes over the drop-in runner's iterations (tools/prof_iter.py, K=1): L2 hit/miss,
# FETCH_SIZE and the SQ wait counters of every learner kernel (per-kernel means:
# tools/pmc_summary.py). Outputs in gpurun_out/pmc_learner/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_learner
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for c in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  K=1 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/p$i -- python3 $R/tools/prof_iter.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O > $O/summary.txt
find $O -name "*_counter_collection.csv" -size +20M -delete
cat $O/summary.txt
