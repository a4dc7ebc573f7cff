set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8.py tests/test_gpu_s8_update.py 2>&1 | tail -1
bash tools/gpu/prof_bench.sh
