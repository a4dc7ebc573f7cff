# per-block cycle accounts of the S8 GEMM (tools/s8_clock.py) and single-problem timings, product
# vs exp/ variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s8clk; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_s8.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PYTHONPATH=.:tools timeout -k 10 200 python -u tools/s8_clock.py exp/s8_clock.so 2>&1 | grep -v amdgpu.ids | tee $O/clock.log | grep -v "last wave"
PYTHONPATH=.:tools timeout -k 10 300 python -u tools/s8_one.py exp/s8_orig.so > $O/one.log 2>&1 || { tail -20 $O/one.log; exit 1; }
tail -1 $O/one.log
