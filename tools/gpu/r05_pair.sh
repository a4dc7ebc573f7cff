# env kernel with two envs per wave: bitwise tests, parity suites, timing vs one env per wave
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pair
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairing.py tests/test_gpu_parity.py tests/test_gpu_trajectory.py tests/test_gpu_terrain.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
LGX_ENVS_PER_WAVE=1 timeout -k 10 200 python -u tools/env_scaling.py > $O/scaling_epw1.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/env_scaling.py > $O/scaling_epw2.txt 2>&1 || exit 1
grep "N=" $O/scaling_epw1.txt; grep "N=" $O/scaling_epw2.txt
