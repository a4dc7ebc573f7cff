set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 400 python -u tools/dbg_s8_steps.py go2_c2 2>&1 | grep -v amdgpu.ids | tail -60
