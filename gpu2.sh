set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pg2 && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/pg2/p1 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg2/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pg2/p2 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg2/p2.log 2>&1
rc=$?
tail -3 $R/gpurun_out/pg2/p2.log
exit $rc
