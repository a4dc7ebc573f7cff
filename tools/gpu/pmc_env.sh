# Env-step kernel PMC on the GPU box (Go2 flat, 4096 envs, tools/env_kernel_driver.py):
# instruction mix / wait fractions, then FETCH_SIZE and WRITE_SIZE in separate passes, and the
# dword-access calibration (tools/calib/hbm_calib). Usage: bash tools/gpu/pmc_env.sh <tag>
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_env_${TAG}_${TASK:-go2}
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/p$i -- python3 $R/tools/env_kernel_driver.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c1 -- $R/tools/calib/hbm_calib > $O/c1.log 2>&1 || { echo "calib fetch failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2 -- $R/tools/calib/hbm_calib > $O/c2.log 2>&1 || { echo "calib write failed"; exit 1; }
cd $R && python3 tools/pmc_env_summary.py $O $TAG
