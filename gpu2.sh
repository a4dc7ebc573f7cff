set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pg && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/bench_mlp.py > $R/gpurun_out/bench_mlp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pg/trace -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pg/p1 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pg/p2 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/pg/p3 -- python3 $R/tools/prof_gemm.py > $R/gpurun_out/pg/p3.log 2>&1
rc=$?
grep -v amdgpu $R/gpurun_out/bench_mlp.log
find $R/gpurun_out/pg -name "*.csv" | head
exit $rc
