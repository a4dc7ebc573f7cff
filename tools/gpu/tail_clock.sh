set -o pipefail
cd $GRAFT_REPO_ROOT
PYTHONPATH=. timeout -k 10 120 python -u tools/tail_clock.py 2>&1 | grep -v amdgpu.ids
LGX_MLP_LIB=legged_gym_custom_amd/lib/dev/liblgx_mlp_clock.so PYTHONPATH=. timeout -k 10 120 python -u tools/tail_clock.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8.py -k "tail or heads" 2>&1 | tail -2
