# PMC passes over runner iterations (tools/prof_iter.py, K=1) for the S8 update kernels: L2,
# FETCH_SIZE, SQ wait / MFMA / LDS counters, TA/TCP stalls (per-kernel means: tools/pmc_summary.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_s8
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for c in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
         "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  K=1 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/p$i -- python3 $R/tools/prof_iter.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O --by-grid > $O/summary.txt
find $O -name "*_counter_collection.csv" -size +20M -delete
cat $O/summary.txt
